set -o pipefail
bash scripts/r4_rt.sh || exit 1
tail -1 gpurun_out/r4/pytest_rt.log
timeout -k 10 300 python -u -c "
import bench, json
print(json.dumps(bench.per_sample_rates(0)))
" > gpurun_out/r4/per_sample.json 2> gpurun_out/r4/per_sample.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/r4/per_sample.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, round(v['us_per_sample'],2), v['real_time_48k'])"
