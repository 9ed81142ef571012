#!/bin/bash
# Builds tools/getrow_bench against the in-tree product library (run from the repo root).
set -e
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude tools/getrow_bench.cpp -o tools/getrow_bench \
  -Lobjectkv_amd -lokv_sst -Wl,-rpath,'$ORIGIN/../objectkv_amd' -ldl
# the same tool against the ablation build (adds the point kernel's phase times)
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude tools/getrow_bench.cpp -o tools/getrow_bench_ablate \
  -Lobjectkv_amd -l:libokv_sst_ablate.so -Wl,-rpath,'$ORIGIN/../objectkv_amd' -ldl
