#!/bin/bash
# One GPU-box session (run through gpurun from the repo root).  Steps, chained so that the first
# failure ends the session, each under its own time limit:
#   tests   pytest -m gpu (whole suite)          bench   bench.py default line (C4, CPU baseline)
#   prof    rocprofv3 kernel trace of bench.py   pmc     FETCH_SIZE / WRITE_SIZE passes -> traffic
#   pmccopy the session's traffic record to profiles/pmc_traffic.json (bench.py reads it)
#   ab:CFG:FIX:LIB_A:LIB_B   alternating kernel-only probes (tools/probe.py) of two libraries
#   matrix  tools/bench_matrix.py (every config)  probe:CFG:FIX  one probe of the working tree
#   ptest:FILE[,FILE]  a subset of the GPU tests    pmcp:CFG:FIX:CTR,CTR  a PMC pass over probe.py (per-kernel)
#   abenv:VAR=VAL   bench.py A/B (tools/ab.sh) without / with VAR=VAL     ablib:LIB_A:LIB_B   the same for two libraries
#   usage: TAG=name [STRICT=1] bash tools/session.sh STEP [STEP ...]   (STRICT: a failing test ends the session)
set -e
TAG=${TAG:-run}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  case "$step" in
    tests)  # (failing tests do not end the session -- pytest exit 1; a crash or a time limit does)
      rc=0
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 900 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1 || rc=$?
      tail -3 "$OUT/gpu_tests.log"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests: exit $rc"; exit 1; fi
      grep -E "^(FAILED|ERROR)" "$OUT/gpu_tests.log" || true
      if [ -n "$STRICT" ] && [ $rc -ne 0 ]; then echo "tests: failures (STRICT): session ends"; exit 1; fi ;;
    checksuite)  # the whole GPU suite on the range-checking build (abl/check.so: tools/build_variant.sh worktree abl/check.so -DCTOK_CHECK)
      rc=0
      CTOK_LIB=$ROOT/abl/check.so timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 900 --timeout-method thread \
        > "$OUT/check_suite.log" 2>&1 || rc=$?
      tail -2 "$OUT/check_suite.log"
      if [ $rc -ne 0 ]; then echo "checksuite: exit $rc"; exit 1; fi ;;
    ptest:*)  # a subset of the GPU tests: ptest:FILE[,FILE...] (paths under tests/)
      rc=0; files=$(echo "${step#ptest:}" | tr , ' ' | sed 's|\([^ ]*\)|tests/\1|g')
      timeout -k 10 900 python -u -m pytest $files -m gpu -v --maxfail=5 --timeout 600 --timeout-method thread \
        > "$OUT/ptest.log" 2>&1 || rc=$?
      tail -3 "$OUT/ptest.log"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ptest: exit $rc"; exit 1; fi
      grep -E "^(FAILED|ERROR)" "$OUT/ptest.log" || true
      if [ -n "$STRICT" ] && [ $rc -ne 0 ]; then echo "ptest: failures (STRICT): session ends"; exit 1; fi ;;
    bench)
      timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -20 "$OUT/bench.log"; exit 1; }
      cat "$OUT/bench.json" ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 "$ROOT/bench.py" --steps 10 --no-cpu-baseline --no-user-facing > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.log") \
        || { tail -20 "$OUT/prof_bench.log"; exit 1; }
      cat "$OUT/prof_bench.json" ;;
    pmc)
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-user-facing --corpus-workers 1 \
        > "$OUT/pmc_fetch.log" 2>&1) || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-user-facing --corpus-workers 1 \
        > "$OUT/pmc_write.log" 2>&1) || { tail -20 "$OUT/pmc_write.log"; exit 1; }
      python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json" c4/10000000 ;;
    pmccopy)  # this session's PMC traffic as the record bench.py reads (hash-matched to libctok.so)
      cp "$OUT/pmc_traffic.json" "$ROOT/profiles/pmc_traffic.json" && echo "pmccopy: profiles/pmc_traffic.json" ;;
    ab:*)
      IFS=: read -r _ cfg fx la lb <<< "$step"
      for i in 1 2 3; do
        for L in "$la" "$lb"; do
          CTOK_LIB=$L timeout -k 10 300 python -u tools/probe.py "$cfg" "$fx" 5 2>>"$OUT/ab_${cfg}.err" > "$OUT/ab_run.txt" \
            || { echo "probe failed: $L"; tail -5 "$OUT/ab_${cfg}.err"; exit 1; }
          grep -E "MB/s|ms_" "$OUT/ab_run.txt" | sed "s|^|$(basename "$L") |" | tee -a "$OUT/ab_${cfg}_${fx}.txt"
        done
      done ;;
    abenv:*)  # bench.py A/B of the working tree's library without / with an environment setting
      L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
      bash tools/ab.sh "$L" "$L,${step#abenv:}" 2>&1 | tee -a "$OUT/abenv.txt" ;;
    ablib:*)  # bench.py A/B of two libraries
      IFS=: read -r _ la lb <<< "$step"
      bash tools/ab.sh "$la" "$lb" 2>&1 | tee -a "$OUT/ablib.txt" ;;
    abpenv:*)  # kernel-only probe A/B of the working tree's library without / with VAR=VAL: abpenv:CFG:FIX:VAR=VAL
      IFS=: read -r _ cfg fx ev <<< "$step"
      L=complexity-tokenizer_amd/complexity_tokenizer/libctok.so
      for i in 1 2 3; do
        for arm in A B; do
          envs=""; [ $arm = B ] && envs=$ev
          env CTOK_LIB=$L $envs timeout -k 10 300 python -u tools/probe.py "$cfg" "$fx" 5 2>/dev/null | grep MB/s \
            | sed "s|^|$arm${envs:+ $envs} |" | tee -a "$OUT/abpenv_${cfg}.txt"
        done
      done ;;
    trace:*)  # kernel trace of tools/probe.py (trace:CFG:FIX[:LIB]) and the last call's timeline
      IFS=: read -r _ cfg fx lib <<< "$step"
      lib=${lib:-complexity-tokenizer_amd/complexity_tokenizer/libctok.so}
      d="$OUT/trace_${cfg}_$(basename "$lib" .so)"
      (cd /tmp && CTOK_LIB="$ROOT/$lib" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- \
        python3 "$ROOT/tools/probe.py" "$cfg" "$fx" 2 > "$d.log" 2>&1) || { tail -20 "$d.log"; exit 1; }
      python3 tools/trace_timeline.py "$d" | tee "$d.txt" ;;
    pmcp:*)  # one PMC pass over tools/probe.py: pmcp:CFG:FIX:COUNTER,COUNTER,... (per-kernel sums)
      IFS=: read -r _ cfg fx ctrs <<< "$step"
      d="$OUT/pmc_${cfg}_$(echo "$ctrs" | tr , _ | cut -c1-40)"
      (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $(echo "$ctrs" | tr , ' ') --output-format csv -d "$d" -o run -- \
        python3 "$ROOT/tools/probe.py" "$cfg" "$fx" 2 > "$d.log" 2>&1) || { tail -20 "$d.log"; exit 1; }
      python3 tools/pmc_sum.py "$d" | tee "$d.txt" ;;
    corpus:*)  # build full-size corpora into the per-box cache (outside any profiler: worker processes)
      timeout -k 10 600 python -u -c "import sys; sys.path.insert(0, '.'); from datagen import cache; cache.build(cache.default_dir(), sys.argv[1].split(','))" \
        "${step#corpus:}" 2>&1 | tee "$OUT/corpus.log" ;;
    avail)  # the PMC counters of this GPU
      (cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1) || true
      grep -c . "$OUT/avail.txt" ;;
    stamps:*)  # k_segment phase stamps (diagnostic build abl/stamps.so, -DCTOK_SEG_STAMPS): stamps:CFG:FIX
      IFS=: read -r _ cfg fx <<< "$step"
      CTOK_LIB=abl/stamps.so CTOK_STAMPS=1 timeout -k 10 300 python -u tools/probe.py "$cfg" "$fx" 2 \
        > "$OUT/stamps_${cfg}.txt" 2>&1 || { tail -5 "$OUT/stamps_${cfg}.txt"; exit 1; }
      grep -E "stamps|MB/s" "$OUT/stamps_${cfg}.txt" | tail -3 ;;
    probe:*)
      IFS=: read -r _ cfg fx <<< "$step"
      timeout -k 10 300 python -u tools/probe.py "$cfg" "$fx" 5 2>&1 | tee -a "$OUT/probe_${cfg}_${fx}.txt" ;;
    trainer)  # GPU trainer vs the C restatement of the reference's per-merge work
      timeout -k 10 600 python -u tools/trainer_timing.py > "$OUT/trainer_timing.json" 2> "$OUT/trainer_timing.log" \
        || { tail -20 "$OUT/trainer_timing.log"; exit 1; }
      cat "$OUT/trainer_timing.json" ;;
    matrix)
      timeout -k 10 900 python -u tools/bench_matrix.py > "$OUT/matrix.json" 2> "$OUT/matrix.log" || { tail -20 "$OUT/matrix.log"; exit 1; }
      tail -5 "$OUT/matrix.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done"
