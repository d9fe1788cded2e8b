set -o pipefail
for d in 0 16 1 2 3 8 24; do echo "== dbg $d"; timeout -k 10 60 tools/halo_bench_diag 128 2 20 sweep0 $d || exit 1; done
