# bench one config under several knob environments: CFG=c3 bash tools/gpu_envexp.sh "ENV1" "ENV2" ...
set -o pipefail
T=${TAG:-envexp}
O=gpurun_out/$T
mkdir -p $O
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --no-cpu-baseline --no-e2e --steps ${STEPS:-10} --warmup 3 > $O/v$i.json 2> $O/v$i.err || { echo "variant '$E' failed"; tail -5 $O/v$i.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['config'];print(sys.argv[2],'|',d['value'],'GB/s',d['ms_per_step'],'ms bails/step',c['exact_path_msgs_per_step'],'ok',c['ok_msgs_rank0'])" $O/v$i.json "$E"
done
