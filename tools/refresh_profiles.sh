# Round artifacts for profiles/: the default bench line, rocprofv3 --kernel-trace --stats of the same
# command (B=32) and of B=1, PMC HBM traffic (separate passes), GEMM vs hipBLASLt.  Writes gpurun_out/refresh/.
set -e
OUT=gpurun_out/refresh
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > $OUT/bench_b32.json 2> $OUT/bench_b32.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof32 -o run -- \
  python bench.py --no-cpu-baseline > $OUT/prof32.log 2>&1
cp $(find $OUT/prof32 -name '*kernel_stats.csv' | head -n 1) $OUT/b32_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof1 -o run -- \
  python bench.py --batch 1 --steps 200 --no-cpu-baseline > $OUT/prof1.log 2>&1
cp $(find $OUT/prof1 -name '*kernel_stats.csv' | head -n 1) $OUT/b1_kernel_stats.csv
OUT=$OUT/pmc bash tools/pmc_bench.sh
python tools/pmc_traffic.py $OUT/pmc $OUT/pmc_traffic_b32.json > $OUT/pmc_traffic.txt
NO_TORCH= SHAPES=fc1,qkv,fc2,proj,sq4k CFGS=-1,9 timeout -k 10 300 python tools/bench_gemm.py > $OUT/gemm_vs_hipblaslt.txt 2>&1
rm -rf $OUT/prof32 $OUT/prof1 $OUT/pmc
