# One parametrised GPU call (replaces the round-4 one-off launchers).
#
#   STAGES="tests bench:C3 bench:C3:fp64 prof:C3 pmc:C3 pmc:C3:fp64 ab py:tools/x.py" \
#   OUT=r5a bash tools/gpu_job.sh
#
# Stages, run in order, each GPU step under its own time limit, chained so
# nothing runs after a failure (outputs under gpurun_out/$OUT):
#   tests            pytest -m gpu over $TESTS (default: tests)
#   bench:CFG[:fp64] one bench.py line (--config CFG, $BENCH_ARGS) -> bench_<cfg>[_fp64].json
#   prof:CFG[:fp64]  rocprofv3 --kernel-trace --stats of that bench command ($PROF_ARGS) -> prof_<cfg>/
#   pmc:CFG[:fp64|:bvh] three PMC passes (FETCH_SIZE / WRITE_SIZE / SQ issue counters;
#                    fp64 adds a fourth: the F64 op counts; bvh = --flags 8, RT_FLAG_NO_BINNING),
#                    one counter group per run -> pmc_<cfg>[_fp64]/ (summarise on the CPU:
#                    python tools/pmc_summary.py gpurun_out/$OUT/pmc_<cfg> <workload key>)
#   ab               interleaved A/B of bench.py over library builds: for $AB_REPS reps,
#                    each variant in $AB_VARIANTS (base = the in-tree librtmi.so, else
#                    tools/ab/<v>.so from tools/build_variant.sh; v@K=V,K2=V2 runs it
#                    with those environment variables, e.g. a RTMI_DIAG build's knobs)
#                    with --config $AB_CONFIG $AB_ARGS; prints ms_per_step / kernel_ms
#   py:SCRIPT[:ARG]  python SCRIPT ARG $PY_ARGS (a measurement tool), stdout -> py_<name>.out
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-job}
mkdir -p $O
K='k_render|k_frame_'
lim() { case $1 in c5*) echo 900;; c4*) echo 400;; *) echo 240;; esac; }
for st in ${STAGES:-tests}; do
  IFS=: read -r kind cfg prec <<< "$st"
  c=$(echo "${cfg:-C3}" | tr A-Z a-z)
  pa=""; sfx=""
  [ "$prec" = fp64 ] && { pa="--precision fp64"; sfx=_fp64; }
  [ "$prec" = bvh ] && { pa="--flags 8"; sfx=_bvh; }   # RT_FLAG_NO_BINNING: the BVH path for every ray
  T=$(lim $c)
  case $kind in
    tests)
      timeout -k 10 1200 python -u -m pytest ${TESTS:-tests} -m gpu -v -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
        || { tail -40 $O/tests.log; exit 1; }
      tail -2 $O/tests.log ;;
    bench)
      timeout -k 10 $T python bench.py --config ${cfg:-C3} $pa ${BENCH_ARGS:-} > $O/bench_$c$sfx.json 2> $O/bench_$c$sfx.err \
        || { tail -20 $O/bench_$c$sfx.err; exit 1; }
      cat $O/bench_$c$sfx.json ;;
    prof)
      timeout -k 10 $T rocprofv3 --kernel-trace --stats -d $O/prof_$c$sfx -o p -f csv -- python3 bench.py --config ${cfg:-C3} $pa \
        --steps ${PROF_STEPS:-5} --warmup 1 --no-cpu ${PROF_ARGS:-} > $O/prof_$c$sfx.json 2> $O/prof_$c$sfx.err || { tail -20 $O/prof_$c$sfx.err; exit 1; }
      cat $O/prof_$c$sfx.json ;;
    pmc)
      P=$O/pmc_$c$sfx
      mkdir -p $P
      S="--config ${cfg:-C3} $pa --steps 2 --warmup 0 --no-cpu --no-extra"
      timeout -s KILL $T rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $P/fetch -o p -f csv -- python3 bench.py $S > /dev/null 2> $P/fetch.err \
        && timeout -s KILL $T rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $P/write -o p -f csv -- python3 bench.py $S > /dev/null 2> $P/write.err \
        && timeout -s KILL $T rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
             --kernel-include-regex "$K" -d $P/sq -o p -f csv -- python3 bench.py $S > /dev/null 2> $P/sq.err \
        || { echo "pmc $c$sfx failed"; tail -5 $P/*.err; exit 1; }
      # float64: the F64 op mix (an F64 VALU instruction issues over 4 cycles, not 2)
      if [ "$prec" = fp64 ]; then
        timeout -s KILL $T rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 \
             --kernel-include-regex "$K" -d $P/f64 -o p -f csv -- python3 bench.py $S > /dev/null 2> $P/f64.err \
          || { echo "pmc $c$sfx f64 failed"; tail -5 $P/f64.err; exit 1; }
      fi
      echo "pmc $c$sfx done" ;;
    ab)
      for i in $(seq ${AB_REPS:-2}); do
        for spec in ${AB_VARIANTS:-base}; do
          v=${spec%%@*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*@}
          tag=$(echo "$spec" | tr '@=,' '___')
          L=""; [ $v != base ] && L=tools/ab/$v.so
          env RTMI_LIB=$L ${envs//,/ } timeout -k 10 $T python bench.py --config ${AB_CONFIG:-C3} --no-cpu \
            ${AB_ARGS:---steps 20 --warmup 3} > $O/ab_${tag}_$i.json 2> $O/ab_${tag}_$i.err || { tail -20 $O/ab_${tag}_$i.err; exit 1; }
          echo "$spec $i $(grep -o '"ms_per_step": [0-9.]*' $O/ab_${tag}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/ab_${tag}_$i.json)"
        done
      done ;;
    py)
      n=$(basename "$cfg" .py)
      timeout -k 10 ${PY_TIMEOUT:-600} python -u $cfg $prec ${PY_ARGS:-} > $O/py_$n.out 2> $O/py_$n.err || { tail -20 $O/py_$n.err; exit 1; }
      tail -${PY_TAIL:-20} $O/py_$n.out ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "gpu_job $OUT ok"
