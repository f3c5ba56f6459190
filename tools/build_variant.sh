#!/bin/bash
# usage: tools/build_variant.sh NAME "-DFLAG=..." — builds tools/bin/libslat_NAME.so (kernel experiments)
set -e
mkdir -p "$(dirname "$0")/bin"
cd "$(dirname "$0")/../sparse-linear-algebra-tests_amd"
make -s
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -I../include -Icsrc $2 -c csrc/slat_api.hip -o /tmp/slat_$1.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../tools/bin/libslat_$1.so /tmp/slat_$1.o build/slat_graph.o build/slat_coo.o build/slat_dense.o build/host_gen.o
