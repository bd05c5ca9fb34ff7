#!/bin/bash
# One GPU-box pass, parameterised (replaces round 1-3's one-off gpu_r*.sh scripts).
#
#   bash tools/gpu.sh <tag> <task> [<task> ...]
#
# tasks (each under its own time limit; the first failure ends the pass):
#   suite                   the whole `pytest -m gpu` suite in one process, then smoke()
#   test:<pytest -k expr>   selected GPU tests
#   bench:<cfg>[:<steps>[:<warmup>]]     one bench.py line (CPU baseline included)
#   quick:<cfg>[:<steps>]   a bench line without the CPU leg
#   trace:<cfg>             rocprofv3 --kernel-trace --stats of the device-resident leg
#   prof:<cfg>[:loc]        kernel trace + separate PMC passes of the same command (FETCH_SIZE, WRITE_SIZE,
#                           the TCC DRAM request counters, SQ stall + L2), summarised and shrunk on the box
#                           (tools/profile_summary.py -> <out>_summary.json, <out>_traffic.json)
#   calib:<mode>:<MB,MB..>  tools/_build/calib_gather --<mode> under a PMC pass of the TCC request counters
#   trloc:<cfg>             rocprofv3 --kernel-trace --stats of a run with the located leg (C5)
#   e2etrace:<cfg>          EDSBWT_TRACE=1 timeline of the end-to-end leg's last calls
#   hostmarks:<cfg>         EDSBWT_TRACE=2 host timeline of the last searches (the fixed per-call cost)
#   rehearse:<N>:<cfg>[:<patterns>]      N ranks on this one GPU over gloo (torchrun)
#   rccl:<cfg>[:<patterns>] one rank through the exchange path over RCCL (bench.py --dist-self)
#   cli:<cfg>               the EDSBWTsearch CLI timed on the config's index and pattern file
#   ab:<cfg>:<VAR=a,VAR2=b>[:<VAR=c>...] A/B bench lines (no CPU leg) under env settings
#   abi:<cfg>:<reps>:<VAR=a,..>:<VAR=b,..>  interleaved A/B: reps x (A, B) device-resident lines (no e2e,
#                           no CPU leg), one summary line each (round 5's one-off r5*.sh passes, folded in)
#   stress:<args>           tools/kdeep_stress.py (every k_deep build, repeated searches) with <args> (',' = ' ')
#   probe3:<lib>[:<waves>]  tools/threeway_probe.py: the README KAT through eds-bwt_amd/_build/<lib> (k_deep's
#                           three-way list start variants), EDSBWT_DEEPQ_WAVES=<waves> (default 1), traced
#   dist:<cfg>              the exchange path with one rank (--dist-self) and the same line without it,
#                           interleaved twice: the step with and without the exchange
# Outputs: gpurun_out/<tag>_<task>*.{json,log}.
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
B0="python3 bench.py --no-cpu --no-e2e --no-located --steps 3 --warmup 1"
fail() { echo "FAIL $1"; tail -30 "$2"; exit 1; }
for task in "$@"; do
  IFS=: read -r kind a b c d <<< "$task"
  tag_a=${a//[^A-Za-z0-9_]/_}
  out=gpurun_out/${TAG}_${kind}${tag_a:+_$tag_a}
  echo "[gpu.sh] $task -> $out ($(date +%T))"
  case $kind in
    suite)
      export EDSBWT_TEST_PROGRESS=$PWD/${out}_progress.log  # (stage lines of the long production tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > ${out}_pytest.log 2>&1 || fail suite ${out}_pytest.log
      tail -2 ${out}_pytest.log
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > ${out}_smoke.log 2>&1 || fail smoke ${out}_smoke.log ;;
    test)
      export EDSBWT_TEST_PROGRESS=$PWD/${out}_progress.log
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$a" > ${out}.log 2>&1 || fail test ${out}.log
      tail -2 ${out}.log ;;
    bench)
      timeout -k 10 900 python bench.py --config ${a:-c3} --steps ${b:-20} --warmup ${c:-3} > ${out}.json 2> ${out}.log || fail bench ${out}.log
      head -c 400 ${out}.json; echo ;;
    quick)
      timeout -k 10 600 python bench.py --no-cpu --config ${a:-c3} --steps ${b:-10} --warmup 2 > ${out}.json 2> ${out}.log || fail quick ${out}.log
      head -c 400 ${out}.json; echo ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${out}_trace -o trace --output-format csv -- $B0 --config ${a:-c3} > ${out}.json 2> ${out}.log || fail trace ${out}.log
      python3 tools/trace_split.py ${out}_trace > ${out}_split.txt 2>&1 || true  # the last search's kernels, before the trace is shrunk
      python3 tools/prof_reduce.py ${out}_trace
      cat ${out}_split.txt ;;
    prof)
      # kernel trace + the four PMC passes of one command, summarised here (profile_summary.py:
      # per-class rocprof averages, DRAM bytes / requests per launch -> <out>_traffic.json) and
      # shrunk (prof_reduce.py) so gpurun_out/ stays under gpurun's copy-back cap
      cfg=${a:-c3}
      # prof:c5:loc profiles the located leg (C5's timed step since round 5) instead of skipping it
      [ "$b" = "loc" ] && B0="python3 bench.py --no-cpu --no-e2e --steps 2 --warmup 1"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${out}_trace -o trace --output-format csv -- $B0 --config $cfg > ${out}_trace.json 2> ${out}_trace.log || fail prof_trace ${out}_trace.log
      grep -v "^[A-Z].*version :\|^Hostname\|^Librccl" ${out}_trace.json | tail -1 > ${out}_bench.json
      timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d ${out}_fetch -o pmc --output-format csv -- $B0 --config $cfg > /dev/null 2> ${out}_fetch.log || fail pmc_fetch ${out}_fetch.log
      timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d ${out}_write -o pmc --output-format csv -- $B0 --config $cfg > /dev/null 2> ${out}_write.log || fail pmc_write ${out}_write.log
      timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d ${out}_tccreq -o pmc --output-format csv -- $B0 --config $cfg > /dev/null 2> ${out}_tccreq.log || fail pmc_tcc ${out}_tccreq.log
      timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum -d ${out}_sq -o pmc --output-format csv -- $B0 --config $cfg > /dev/null 2> ${out}_sq.log || fail pmc_sq ${out}_sq.log
      python3 tools/prof_reduce.py ${out}_trace ${out}_fetch ${out}_write ${out}_tccreq ${out}_sq
      python3 tools/profile_summary.py ${out}_trace ${out}_fetch ${out}_write ${out}_bench.json ${out}_summary.json --tcc ${out}_tccreq \
          --traffic ${out}_traffic.json --source "tools/gpu.sh prof:$cfg (rocprofv3 --pmc passes of $B0 --config $cfg)" > /dev/null || fail prof_summary ${out}_trace.log
      tail -c 300 ${out}_traffic.json; echo ;;
    calib)
      # tools/_build/calib_gather --<a> <sizes, comma-separated> under one PMC pass of the TCC request
      # counters (requests per access of a shape: random 16-B stores, large-table gathers)
      timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_DRAM_32B_sum -d ${out}_pmc -o pmc --output-format csv -- tools/_build/calib_gather --$a ${b//,/ } > ${out}.json 2> ${out}.log || fail calib ${out}.log
      python3 tools/prof_reduce.py ${out}_pmc
      cat ${out}.json; find ${out}_pmc -name "*counter_collection.csv" -exec cat {} \; ;;
    trloc)
      # kernel trace of the located leg (C5: every pattern searched WITH locate in record-budget chunks)
      # beside one count-only step; the per-chunk split is in the bench line's `located`
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d ${out}_trace -o trace --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 1 --warmup 0 --config ${a:-c5} > ${out}.json 2> ${out}.log || fail trloc ${out}.log
      python3 tools/prof_reduce.py ${out}_trace
      find ${out}_trace -name "*kernel_stats.csv" -exec head -30 {} \; ;;
    e2etrace)
      # the end-to-end leg's pipeline timeline (EDSBWT_TRACE=1: upload / search / download marks per chunk)
      EDSBWT_TRACE=1 timeout -k 10 300 python3 bench.py --no-cpu --no-device --no-located --steps 3 --warmup 1 --config ${a:-c2} > ${out}.json 2> ${out}.log || fail e2etrace ${out}.log
      grep -E "\] t +[0-9.]+ ms" ${out}.log | tail -40 > ${out}_tail.txt || true; rm -f ${out}.log; cat ${out}_tail.txt ;;
    hostmarks)
      # host time of every launch inside each search (EDSBWT_TRACE=2) of a short device-resident run
      EDSBWT_TRACE=2 timeout -k 10 300 $B0 --config ${a:-c2} > ${out}.json 2> ${out}.log || fail hostmarks ${out}.log
      tail -120 ${out}.log > ${out}_tail.txt; rm -f ${out}.log; tail -60 ${out}_tail.txt ;;
    rehearse)
      n=${a:-2}; cfg=${b:-c4}
      timeout -k 10 1100 python bench.py --gpus $n --config $cfg --steps 3 --warmup 1 --dist-backend gloo ${c:+--patterns $c} > ${out}_${b}.json 2> ${out}_${b}.log || fail rehearse ${out}_${b}.log
      head -c 400 ${out}_${b}.json; echo ;;
    rccl)
      # the N>1 exchange path with one rank on this GPU: process group over RCCL, sizes all-gathered,
      # counts gathered from the engine's device mirror (bench.py --dist-self)
      timeout -k 10 600 python bench.py --dist-self --config ${a:-c3} --steps 5 --warmup 2 --no-cpu ${b:+--patterns $b} > ${out}.json 2> ${out}.log || fail rccl ${out}.log
      head -c 400 ${out}.json; echo ;;
    cli)
      timeout -k 10 900 python tools/cli_timing.py --config ${a:-c3} > ${out}.json 2> ${out}.log || fail cli ${out}.log
      cat ${out}.json ;;
    ab)
      cfg=${a:-c3}; i=0
      for spec in "$b" "$c" "$d"; do
        [ -z "$spec" ] && continue
        i=$((i+1))
        env ${spec//,/ } timeout -k 10 600 python bench.py --no-cpu --no-located --config $cfg --steps 5 --warmup 2 > ${out}_$i.json 2> ${out}_$i.log || fail ab ${out}_$i.log
        python3 -c "import json;d=json.load(open('${out}_$i.json'));r=d.get('device_resident',{});e=d.get('e2e') or {};print('$spec', d['value'], d['ms_per_step'], r.get('kernel_ms_per_step'), 'e2e median', e.get('ms_wall_median'))"
      done ;;
    abi)
      cfg=${a:-c3}; reps=${b:-3}
      for k in $(seq 1 $reps); do
        for spec in "$c" "$d"; do
          [ -z "$spec" ] && continue
          sid=${spec//[^A-Za-z0-9]/_}
          env ${spec//,/ } timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-located --config $cfg --steps 20 --warmup 3 > ${out}_${k}_${sid}.json 2>> ${out}.log || fail abi ${out}.log
          python3 -c "import json;d=json.load(open('${out}_${k}_${sid}.json'));print('$k', '$spec', d['ms_per_step'], d['device_resident']['kernel_ms_per_step'])" | tee -a ${out}_summary.txt
        done
      done ;;
    stress)
      timeout -k 10 900 python3 tools/kdeep_stress.py ${a//,/ } > ${out}.json 2> ${out}.log || fail stress ${out}.log
      tail -5 ${out}.json ;;
    dist)
      cfg=${a:-c3}
      for k in 1 2; do
        timeout -k 10 600 python bench.py --dist-self --config $cfg --steps 20 --warmup 3 --no-cpu > ${out}_self_$k.json 2>> ${out}.log || fail dist ${out}.log
        timeout -k 10 600 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > ${out}_plain_$k.json 2>> ${out}.log || fail dist ${out}.log
        python3 -c "
import json
a=json.load(open('${out}_self_$k.json'));b=json.load(open('${out}_plain_$k.json'))
print('$k', 'exchange', a['ms_per_step'], a['e2e']['per_rank_search_exchange_ms'], 'plain', b['ms_per_step'], b['e2e']['per_rank_search_exchange_ms'])" | tee -a ${out}_summary.txt
      done ;;
    probe3)
      # k_deep's three-way list start: the README KAT through the library named by
      # <a> (a file under eds-bwt_amd/_build/), unbounded k_deep build, traced; one process
      EDSBWT_LIB=$PWD/eds-bwt_amd/_build/${a:-libedsbwt_3way.so} EDSBWT_DEEPQ_WAVES=${b:-1} EDSBWT_TRACE=1 EDSBWT_PATH_TAGS=1 \
        timeout -k 10 120 python3 tools/threeway_probe.py > ${out}_${b:-1}.json 2> ${out}_${b:-1}.log || fail probe3 ${out}_${b:-1}.log
        python3 -c "import json;d=json.load(open('${out}_${b:-1}.json'));print(d['lib'][-24:], d['oracle_counts'], [(r['kw'], r.get('counts', r.get('error'))) for r in d['runs']]);[print(x) for x in d.get('kdeep_dump', [])]" ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
echo "[gpu.sh] EXIT 0 ($(date +%T))"
