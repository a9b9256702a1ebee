set -o pipefail
for g in 1 2 3 4 6; do echo "gpx $g"; SYZCOV_PRIO_GPX=$g timeout -k 10 120 python3 bench.py --workload prio --no-cpu | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['phases_ms'], round(d['roofline']['frac'],4))" || exit 1; done
