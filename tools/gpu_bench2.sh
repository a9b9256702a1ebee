#!/bin/bash
# corpus bench: key mode (default) and window mode, no CPU leg
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/b
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/b/keys.json 2> gpurun_out/b/keys.err || { tail -20 gpurun_out/b/keys.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b/keys.json'));print('keys', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['roofline'].get('peak_measured'))"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-universe > gpurun_out/b/win.json 2> gpurun_out/b/win.err || { tail -20 gpurun_out/b/win.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b/win.json'));print('window', d['ms_per_step'], d['phases_ms'], d['roofline']['frac'])"
