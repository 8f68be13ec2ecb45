#!/bin/bash
# round 5: layout probe (product kernels over three HBM layouts), then the
# default bench line (host_path.rows_call: the writer / reader call shapes)
set -o pipefail
out=gpurun_out/r05d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/probe_layout.py > $out/probe_layout.txt 2>&1 || { tail -20 $out/probe_layout.txt; exit 1; }
cat $out/probe_layout.txt
timeout -k 10 600 python3 -u bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 2; }
python3 -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac']); print(json.dumps(d['host_path']['rows_call'], indent=1))
print(json.dumps(d.get('ranks')), d.get('distinct_gpus'))
for c in d.get('cpu_baseline_configs', []): print(c['config'], json.dumps(c['legs']))"
