set -e
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
for v in old nobmax s64x4nob; do
  echo -n "$v "; SLAT_LIB_PATH=tools/var/libslat_$v.so timeout -k 10 120 python3 tools/c4_eighth.py
done; done
