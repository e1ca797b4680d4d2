set -o pipefail
export TMPDIR=/tmp
for v in fused unfused; do
  out=gpurun_out/r03_t14/$v; mkdir -p $out
  if [ $v = unfused ]; then export SCA_FUSE_LN=0 SCA_FUSE_LNB=0; else unset SCA_FUSE_LN SCA_FUSE_LNB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $out/bench.log 2>&1 || exit 1
  f=$(ls $out/*kernel_trace.csv | head -1); python3 tools/timeline.py $f > $out/timeline.txt; head -14 $out/timeline.txt
done
