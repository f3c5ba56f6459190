#!/bin/bash
# usage: tools/build_variant.sh NAME SRC "-DFLAG=..." — builds tools/bin/libslat_NAME.so with SRC
# (e.g. slat_fused) compiled with the extra flags and the tree's other objects (kernel experiments)
set -e
mkdir -p "$(dirname "$0")/bin"
cd "$(dirname "$0")/../sparse-linear-algebra-tests_amd"
make -s
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -I../include -Icsrc $3 -c csrc/$2.hip -o /tmp/slat_$1.o
objs=""
for o in $(sed -n "s/^libslat.so: //p" Makefile); do [ "$o" = "build/$2.o" ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../tools/bin/libslat_$1.so /tmp/slat_$1.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
