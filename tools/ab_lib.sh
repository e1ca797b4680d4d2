# bench A/B of the in-tree library against scattennet_amd/libscatten_hip_prev.so (same ABI), alternating
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in new prev; do
    if [ $v = prev ]; then export SCA_LIB_PATH=scattennet_amd/libscatten_hip_prev.so; else unset SCA_LIB_PATH; fi
    timeout -k 10 200 python bench.py --steps ${STEPS:-100} --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit 1
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/ab_$v.log)"
  done
done
