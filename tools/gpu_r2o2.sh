set -o pipefail
for ch in 1 2 4; do
timeout -k 10 300 env DG_E2E_CHUNKS=$ch python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/r2o2_$ch.json 2> gpurun_out/r2o2_$ch.err || { tail -20 gpurun_out/r2o2_$ch.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r2o2_$ch.json').read().strip().splitlines()[-1]);e=d['e2e_host'];print($ch, e['value'], e['ms'])"
done
