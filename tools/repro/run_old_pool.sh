#!/bin/bash
# The round-1 library at 37c5f55^ (all device memory from the stream-ordered pool) on the generator
# sequence that showed the lost writes (tools/check_generators.py: 30^3 then 100^3 on one context).
# tools/repro/old37/ is built locally from that commit (git worktree + make; not committed).
cd "$(dirname "$0")/old37" && SLAT_LIB_PATH=$PWD/libslat_pool.so PYTHONPATH=$PWD python3 -u check_generators.py
