#!/bin/bash
# per-launch host cost: the runtime alone (launch_latency.hip, built here), the library's host split
# of a headline call (variant library, SLAT_HOST_CLOCK), and the headline per call with device vs
# host kernel-argument buffers
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05launch}; mkdir -p $OUT
timeout -k 10 120 /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/repro/launch_latency.hip -o $OUT/ll > $OUT/build.log 2>&1 || { tail $OUT/build.log; exit 1; }
timeout -k 10 120 $OUT/ll > $OUT/ll.txt 2>&1 || { tail $OUT/ll.txt; exit 1; }
cat $OUT/ll.txt
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 $OUT/ll > $OUT/ll_hostk.txt 2>&1 || { tail $OUT/ll_hostk.txt; exit 1; }
echo "HIP_FORCE_DEV_KERNARG=0:"; cat $OUT/ll_hostk.txt
SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_HOST_CLOCK=1 timeout -k 10 120 python3 tools/prof_head.py 600 > $OUT/hc.txt 2>&1 || { tail $OUT/hc.txt; exit 1; }
tail -3 $OUT/hc.txt
for i in 1 2; do
timeout -k 10 120 python3 tools/prof_head.py 400 2>&1 | tail -1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python3 tools/prof_head.py 400 2>&1 | tail -1 | sed 's/^/hostk /'
done
