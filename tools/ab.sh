# A/B bench runs, alternated 3x: tools/ab.sh "ENV=.. ENV2=.." "ENV=.." ... (quoted env lists)
mkdir -p gpurun_out
i=0
for cfg in "$@" "$@" "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --steps ${AB_STEPS:-100} --no-cpu-baseline > gpurun_out/ab$i.log 2>&1 || exit $?
  echo "[$cfg] $(grep -o '"value": [0-9.]*' gpurun_out/ab$i.log)"
done
