#!/bin/bash
# Round-4 GPU check, in stages (each under its own time limit; stops at the first failure):
#   tests   all -m gpu tests
#   bench   the driver-shaped bench line (N = 1) and the N > 1 code path on a one-rank group
#           (--sharded, with the configs[3] strong leg)
#   ab      bench.py A/B of the variant libraries listed in $VARS (var/*.so, see mkvar.sh)
#   abenv   bench.py A/B over environment settings ($AB_ENVS)
#   nat     natural 8192^2 encodes at -s1..-s4 ($NAT_PROF_SPEEDS; one image at a time) + rocprofv3 kernel stats per speed
#   inflight  bench.py (100 steps) over images in flight x GPU_MAX_HW_QUEUES ($INFLIGHT: "D:Q ..."; Q 0 =
#           the bench default, hw_queues_for(D))
#   noix    no-index decode (synthetic + natural, one image at a time) and the no-index pipeline leg,
#           once per environment setting in $NOIX_ENVS ("A=1,B=2 C=3 ..."; "-" = defaults)
#   natab   natural 8192^2 encodes at the speeds in $NAT_SPEEDS once per setting in $NAT_ENVS
#   trace   rocprofv3 --kernel-trace of a 40-step bench run (20 in flight): every dispatch's start / end
#   pmc     rocprofv3 --pmc passes over bench.py --pmc-probe (one image encoded + decoded twice), one
#           pass per ';'-separated counter set in $PMC_SETS (default: the SQ instruction / wait mix);
#           $PMC_PROG replaces the probe (e.g. "tools/scripts/natural_prof.py 8192 0 1")
# usage: round_check.sh OUTDIR stage...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for st in "$@"; do
  case $st in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $O/gputests.log 2>&1 \
        || { tail -30 $O/gputests.log; exit 1; }
      tail -2 $O/gputests.log ;;
    bench)
      timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
      timeout -k 10 240 python -u bench.py --sharded --steps 20 --warmup 5 > $O/sharded.json 2> $O/sharded.err \
        || { tail $O/sharded.err; exit 1; }
      python3 - $O <<'PY'
import json, sys
for f in ("bench", "sharded"):
    d = json.loads(open(sys.argv[1] + "/%s.json" % f).read().strip().splitlines()[-1])
    det = d["detail"]
    print(f, d["value"], {k: det.get(k) for k in ("bit_exact_vs_reference", "slot_files_bit_exact", "no_index_decode_MBps",
          "no_index_pipeline_MBps", "natural_s0_single_MBps", "strong_16384_MBps", "strong_16384_bit_exact_vs_reference")})
PY
      ;;
    ab)
      B="--no-legs --no-pmc --no-cpu-baseline --no-config2"
      for v in base $VARS; do
        n=$(basename $v .so)
        if [ "$v" = base ]; then unset HOH_LIB; else export HOH_LIB=$GRAFT_REPO_ROOT/$v; fi
        timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 $B > $O/ab_${n}.json 2> $O/ab_err || { tail $O/ab_err; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/ab_${n}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', d['value'], r['avg_launch_ms'], r['avg_launch_ms_under_load'], d['detail']['bit_exact_vs_reference'], d['detail']['slot_files_bit_exact'])"
      done
      unset HOH_LIB ;;
    abenv)
      # bench.py A/B over environment settings ($AB_ENVS: "A=1,B=2 C=3 ..."; "-" = defaults)
      B="--no-legs --no-pmc --no-cpu-baseline --no-config2"
      for ev in ${AB_ENVS:--}; do
        E=""; [ "$ev" != "-" ] && E=$(echo $ev | tr ',' ' ')
        n=$(echo $ev | tr ',=' '__')
        timeout -k 10 200 env $E python -u bench.py --steps 100 --warmup 5 $B > $O/abe_${n}.json 2> $O/ab_err || { tail $O/ab_err; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/abe_${n}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('[$ev]', d['value'], r['avg_launch_ms'], r['avg_launch_ms_under_load'], d['detail']['bit_exact_vs_reference'], d['detail']['slot_files_bit_exact'])"
      done ;;
    inflight)
      B="--no-legs --no-pmc --no-cpu-baseline --no-config2"
      for dq in ${INFLIGHT:-16:0 20:0 24:0 28:0 32:0 40:0 24:24 28:28}; do
        d=${dq%:*}; q=${dq#*:}
        timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --inflight $d --hw-queues $q $B > $O/if_${d}_${q}.json 2> $O/if_err \
          || { tail $O/if_err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/if_${d}_${q}.json')); print('inflight $d queues $q', d['value'], d['detail']['latency_ms_enc'], d['detail']['latency_ms_dec'])"
      done ;;
    noix)
      for ev in ${NOIX_ENVS:--}; do
        E=""; [ "$ev" != "-" ] && E=$(echo $ev | tr ',' ' ')
        for kind in synth natural; do
          timeout -k 10 120 env $E python3 tools/scripts/noix_bench.py $kind 8192 5 > $O/noix.txt 2>&1 || { tail $O/noix.txt; exit 1; }
          echo "[$ev] $(grep no-index $O/noix.txt | cut -c1-160)"
        done
        timeout -k 10 200 env $E python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-config2 > $O/noixb.json 2> $O/noixb.err \
          || { tail $O/noixb.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/noixb.json').read().strip().splitlines()[-1])['detail']; print('[$ev] pipeline', d.get('no_index_pipeline_MBps'), d.get('no_index_pipeline_lossless'), 'single', d.get('no_index_decode_MBps'))"
      done ;;
    natab)
      for ev in ${NAT_ENVS:--}; do
        E=""; [ "$ev" != "-" ] && E=$(echo $ev | tr ',' ' ')
        for sp in ${NAT_SPEEDS:-3 4}; do
          timeout -k 10 300 env $E python3 tools/scripts/natural_prof.py 8192 $sp 2 > $O/natab.txt 2>&1 || { tail $O/natab.txt; exit 1; }
          echo "[$ev] $(grep ^natural $O/natab.txt)"
        done
      done ;;
    trace)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run \
        -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-legs --no-pmc --no-cpu-baseline --no-config2) \
        > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
      ls -la $(find $O/trace -name "*kernel_trace.csv") ;;
    pmc)
      SETS=${PMC_SETS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAVES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE"}
      k=0
      IFS=';' read -ra SA <<< "$SETS"
      for set in "${SA[@]}"; do
        k=$((k+1))
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc$k -o p \
          -- python3 $GRAFT_REPO_ROOT/${PMC_PROG:-bench.py --pmc-probe}) > $O/pmc$k.log 2>&1 || { tail -5 $O/pmc$k.log; exit 1; }
      done
      python3 tools/scripts/pmc_summary2.py $O/pmc* > $O/pmc_summary.txt; cat $O/pmc_summary.txt ;;
    nat)
      for sp in ${NAT_PROF_SPEEDS:-1 2 3 4}; do
        (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/nat$sp -o run \
          -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 $sp 2) > $O/nat$sp.txt 2>&1 || { tail $O/nat$sp.txt; exit 1; }
        grep "^natural" $O/nat$sp.txt
        python3 tools/scripts/kstats.py $O/nat$sp 6 2>/dev/null || head -7 $O/nat$sp/run_kernel_stats.csv | cut -d, -f1-4
      done ;;
  esac
done
