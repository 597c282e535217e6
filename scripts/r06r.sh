# round 6, pass r: the final tree's bench lines — default (K = 1,000) and the driver's form (K = 20)
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 600 python -u bench.py --detail $O/bench_detail_n1.json > $O/bench_n1.json 2> $O/bench_n1.err && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --detail $O/bench_detail_n1_k20.json > $O/bench_n1_k20.json 2> $O/bench_n1_k20.err && \
python3 scripts/dispatch_times_summary.py $O/bench_detail_n1.json --md $O/dispatch_times.md > /dev/null && \
python3 -c "
import json
for f in ('bench_n1', 'bench_n1_k20'):
    d = json.load(open('$O/' + f + '.json'))
    r = d['roofline']
    print(f, d['value'] / 1e9, d['ms_per_step'] * 1e3, r['frac'], r.get('frac_profile'), {k: v.get('value') for k, v in d['configs'].items()})
"
