#!/bin/bash
# rocprofv3 evidence for the bench lines (run on the GPU box from the repo root):
#   corpus C3 (the headline) and C2 (the sub-record): kernel trace + stats, and
#     FETCH_SIZE / WRITE_SIZE passes over one step -> per-phase HBM bytes
#   canon wave counters (tools/kbench.py step --keys, one C2 step)
#   newcov C5 (steady state) and dedup: trace + stats, FETCH / WRITE of the
#     timed batches only;  prio C4: trace + stats
#   -> OUT/traffic.json {"C3": phases, "C2": phases, "newcov": ..., "dedup": ...}
# Counters are never combined with tracing; each pass is its own run within the
# per-block limits (MI355X_MICROARCH.md, HBM / rocprofv3).
#   rank: rank 0's share of C3 over 8 GPUs (bench --rank-share-only): trace +
#     FETCH / WRITE of its one timed step -> traffic.json["C3R8"]
#   prio_mfma: SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES of the C4 GEMMs
#     (positional and dense) -> OUT/prio_mfma_pmc.txt
#   usage: tools/profile.sh OUT [parts: corpus rank canon newcov newcov_early dedup groups prio prio_mfma]
set -o pipefail
export TMPDIR=/tmp
o=${1:-gpurun_out/prof}; shift
parts=${*:-corpus rank canon newcov newcov_early dedup groups prio prio_mfma}
mkdir -p $o
B="python3 bench.py --no-cpu --no-c2 --no-dropin --no-rank-share"
has() { case " $parts " in *" $1 "*) return 0;; esac; return 1; }
pmc_pair() {  # name, step kernel ("" = bin_kernel), last-N ("" = all steps), bench args...
  local name=$1 sk=$2 last=$3; shift 3
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${name}_fetch -o run -- "$@" > $o/${name}_f.log 2>&1 || { tail -5 $o/${name}_f.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${name}_write -o run -- "$@" > $o/${name}_w.log 2>&1 || { tail -5 $o/${name}_w.log; exit 1; }
  python3 tools/traffic.py $o/${name}_fetch $o/${name}_write $o/traffic_${name}.json $sk $last > /dev/null && cat $o/traffic_${name}.json
}
trace() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${name}_trace -o run -- "$@" > $o/${name}_trace.log 2>&1 || { tail -20 $o/${name}_trace.log; exit 1; }
  python3 tools/trace_summary.py $o/${name}_trace > $o/${name}_summary.txt && head -16 $o/${name}_summary.txt
}
if has corpus; then
  trace C3 $B --steps 5 --warmup 2
  pmc_pair C3 "" "" $B --steps 1 --warmup 0
  trace C2 $B --global-inputs 1000000 --steps 10 --warmup 2
  pmc_pair C2 "" "" $B --global-inputs 1000000 --steps 1 --warmup 0
  trace C2X $B --global-inputs 1000000 --x86 --steps 10 --warmup 2
  pmc_pair C2X "" "" $B --global-inputs 1000000 --x86 --steps 1 --warmup 0
fi
if has rank; then  # the 8-GPU step's per-rank share (its timed step: the last bin_kernel on)
  trace C3R8 $B --rank-share-only --no-order-parts --steps 5 --warmup 2
  python3 tools/trace_timeline.py $o/C3R8_trace bin_kernel 0 > $o/C3R8_timeline.txt
  pmc_pair C3R8 bin_kernel 1 $B --rank-share-only --no-order-parts --steps 1 --warmup 0
fi
if has canon; then
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
             "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $o/pmc$i -o run -- python3 tools/kbench.py step --keys --reps 1 > $o/pmc$i.log 2>&1 || { tail -3 $o/pmc$i.log; echo "pmc pass $i failed"; exit 1; }
  done
  python3 tools/pmc_summary.py $o > $o/pmc_summary.txt 2>&1; grep -A18 "canon_key_kernel<32" $o/pmc_summary.txt | head -20
fi
if has newcov; then
  N="$B --workload newcov --no-early --steps 10 --warmup 3"
  trace newcov $N
  python3 tools/trace_last.py $o/newcov_trace newcov_own 10 > $o/newcov_timed_summary.txt && head -14 $o/newcov_timed_summary.txt
  pmc_pair newcov newcov_own 10 $N
fi
if has newcov_early; then  # the early regime: 32 history batches, every record still new
  E="$B --workload newcov --history 32 --steps 10 --warmup 3"
  trace newcov_early $E
  python3 tools/trace_last.py $o/newcov_early_trace newcov_own 10 > $o/newcov_early_timed_summary.txt && head -14 $o/newcov_early_timed_summary.txt
  pmc_pair newcov_early newcov_own 10 $E
fi
if has dedup; then
  D="$B --workload dedup --steps 10 --warmup 3"
  trace dedup $D
  python3 tools/trace_last.py $o/dedup_trace "narrow_kernel<4>" 10 > $o/dedup_timed_summary.txt
  pmc_pair dedup "narrow_kernel<4>" 10 $D
fi
if has groups; then  # Manager.minimizeCorpus from host buffers (C2 in 293 call groups)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/groups_trace -o run -- python3 tools/kbench.py groups --reps 2 > $o/groups_trace.log 2>&1 || { tail -20 $o/groups_trace.log; exit 1; }
  python3 tools/trace_summary.py $o/groups_trace > $o/groups_summary.txt && head -24 $o/groups_summary.txt
  python3 tools/trace_last.py $o/groups_trace group_min_kernel 1 > $o/groups_last_call.txt; head -30 $o/groups_last_call.txt
fi
if has prio; then
  trace prio $B --workload prio --steps 10 --warmup 3
  trace prio_dense $B --workload prio --prio-dense --steps 10 --warmup 3
fi
if has prio_mfma; then  # MFMA utilisation of the contraction (one pass per mode)
  for m in pos dense; do
    a=""; [ $m = dense ] && a="--prio-dense"
    timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $o/pmcprio_$m -o run -- $B --workload prio $a --steps 3 --warmup 1 > $o/pmcprio_$m.log 2>&1 || { tail -3 $o/pmcprio_$m.log; echo "prio pmc $m failed"; exit 1; }
  done
  python3 tools/mfma_summary.py $o/pmcprio_pos $o/pmcprio_dense > $o/prio_mfma_pmc.txt; cat $o/prio_mfma_pmc.txt
fi
python3 - $o <<'PY'
import glob, json, os, sys
o = sys.argv[1]
out = {}
for f in sorted(glob.glob(os.path.join(o, "traffic_*.json"))):
    out[os.path.basename(f)[8:-5]] = json.load(open(f))
out["_source"] = ("rocprofv3 --pmc FETCH_SIZE (x2, MI355X_MICROARCH.md) / WRITE_SIZE passes over "
                  "bench.py (C3 / C2: one step; newcov / dedup: the 10 timed batches), "
                  "tools/profile.sh -> tools/traffic.py")
json.dump(out, open(os.path.join(o, "traffic.json"), "w"), indent=1, sort_keys=True)
PY
echo profile_done
