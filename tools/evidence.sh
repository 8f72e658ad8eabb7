#!/bin/bash
# The one recipe behind the numbers in DESIGN.md §5 and profiles/ (run on the GPU box through
# gpurun, from the repository root).  Usage:
#
#   tools/evidence.sh TAG STEP [STEP ...]
#
# Every step writes gpurun_out/TAG_<step>.* and ends the script at the first failure other
# than failing tests (pytest exit 1), so a crash, abort or time limit is never followed by
# more GPU work.  Steps:
#   suite        pytest -m gpu (one process) and smoke()
#   bench        the default bench line (python bench.py)
#   stats        rocprofv3 --kernel-trace --stats of a 20-step bench run (kernel averages)
#   traffic      two PMC passes (FETCH_SIZE, WRITE_SIZE) over a 2-step bench run, reduced by
#                tools/pmc_traffic.py (gfx950 x2 read correction) into TAG_traffic.json
#   gensq        SQ counters of the generator (one 32 768 x 1e4 x 64 launch after a warm-up)
#   genlds       LDS counters of the generator (instructions, bank conflicts, active cycles)
#   genab        generator A/B over tuning builds (GENAB=main,kw8: tools/gen_lib_ab.py)
#   genldsab     LDS counters of each tuning build (GENAB_LDS="main kw8", OCX_LIB)
#   pipeab       FTRL/FTL kernel A/B over tuning builds (PIPEAB=main,pys,...: tools/pipe_lib_ab.py)
#   alg          FTRL / FTL kernel times on the resident batches (tools/alg_probe.py)
#   algsq        SQ counters of the pipelined FTRL / FTL kernels (tools/alg_sq.py, few-wave batch)
#   overlap      tools/overlap_probe.py (sub-batch overlap of generation and FTRL vs sequential)
#   pipetraffic  FETCH_SIZE / WRITE_SIZE of the overlapped pipeline's kernels (tools/pipe_traffic.py)
#   overlaptrace rocprofv3 --kernel-trace of the overlapped pipeline (concurrency evidence)
#   trail        tools/trail_probe.py (trailing pipeline vs sequential: configs[4], configs[3] T=1e5)
#   trailtrace   rocprofv3 --kernel-trace of the trailing pipeline on the T = 1e5 case
#   trailtraffic FETCH_SIZE / WRITE_SIZE of the trailing pipeline's kernels (tools/trail_traffic.py)
#   genwaves     tools/genwaves_probe.py (generator time and SQ counters vs waves per SIMD, d = 1024
#                and d = 64 forms), three PMC passes summed per launch size
#   config4      tools/config4_probe.py (configs[4]: gen / FTRL per batch size, batches of whole waves)
#   gpusub       a subset of pytest -m gpu (GPUSUB='-k expr' or file names)
#   genscale     tools/genscale_probe.py (d = 1024 generator time vs streams per SIMD)
#   cumask       tools/cumask_map (CU-mask placement) and tools/cumask_probe.py (CU-split overlap)
#   config3      tools/perf_extra.py config3 (configs[2]: FTRL vs exact FTL, generation included)
#   sweep        tools/perf_extra.py sweep config4 (configs[3] g(T) sweep and configs[4])
#   layout       tools/e2e_layout.py (generation + FTRL by lane layout, d = 64)
#   smalld       tools/gt_small_d.py (g(T) layouts for 4 <= d < 64)
#   smallpipe    tools/small_pipe_probe.py (configs[1]'s d = 16 / 32 g(T): sequential vs pipeline)
#   smart        tools/smart_probe.py (SMART kernels)
#   twin         tools/twin32_probe.py (the float32 twin's timings)
#   exact        tools/exact_probe.py (the general exact comparator)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG="$1"
shift
O="$R/gpurun_out/$TAG"
fail() { echo "$1 failed (rc $2)"; exit "$2"; }
for step in "$@"; do
  case "$step" in
  suite)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "${O}_suite.log" 2>&1
    rc=$?; tail -1 "${O}_suite.log"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || fail suite $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "${O}_smoke.log" 2>&1 || fail smoke $?
    tail -1 "${O}_smoke.log" ;;
  bench)
    timeout -k 10 600 python bench.py > "${O}_bench.log" 2>&1 || fail bench $?
    grep '^{' "${O}_bench.log" > "${O}_bench.json"; cut -c1-300 "${O}_bench.json" ;;
  stats)
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "${O}_stats" -o s --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 --two-pass-steps 0 > "${O}_stats.log" 2>&1) || fail stats $?
    head -6 "${O}_stats/s_kernel_stats.csv" | cut -c1-160 ;;
  traffic)
    for C in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "${O}_pmc_$C" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-seconds 0 --two-pass-steps 0 --e2e-steps 1 > "${O}_pmc_$C.log" 2>&1) || fail "pmc $C" $?
    done
    python tools/pmc_traffic.py --fetch "${O}_pmc_FETCH_SIZE" --write "${O}_pmc_WRITE_SIZE" --kernel "ocx_alg_pipe_kernel<8, 8, 9," --label ocx_alg_pipe_kernel --B 32768 --T 10000 --d 64 --P 8 --passes 1 --out "${O}_traffic.json" > /dev/null || fail traffic $?
    head -c 600 "${O}_traffic.json"; echo ;;
  gensq)
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "${O}_gensq" -o sq -- python3 "$R/tools/gen_only.py" 32768 10000 64 2 128 > "${O}_gensq.log" 2>&1) || fail gensq $?
    python tools/pmc_summary.py --kernel gen_wave "${O}_gensq" ;;
  genlds)
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d "${O}_genlds" -o lds -- python3 "$R/tools/gen_only.py" 32768 10000 64 2 128 > "${O}_genlds.log" 2>&1) || fail genlds $?
    python tools/pmc_summary.py --kernel gen_wave "${O}_genlds" ;;
  genab)
    # tuning builds tune_r04/libocx_{kw1,kw8}.so (_build.build_variant): bit identity + time
    timeout -k 10 500 python -u tools/gen_lib_ab.py "${GENAB:-main,kw8}" > "${O}_genab.jsonl" 2> "${O}_genab.err" || fail genab $?
    cut -c1-200 "${O}_genab.jsonl" ;;
  genldsab)
    for v in ${GENAB_LDS:-main kw8}; do
      (cd /tmp && export TMPDIR=/tmp && OCX_LIB="$( [ "$v" = main ] && echo "$R/online_convex_optimization_amd/libocx.so" || echo "$R/tune_r04/libocx_$v.so" )" timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d "${O}_genlds_$v" -o lds -- python3 "$R/tools/gen_only.py" 32768 10000 64 2 128 > "${O}_genlds_$v.log" 2>&1) || fail "genlds $v" $?
      python tools/pmc_summary.py --kernel gen_wave "${O}_genlds_$v"
    done ;;
  pipeab)
    timeout -k 10 500 python -u tools/pipe_lib_ab.py "${PIPEAB:-main,pys,pftl}" > "${O}_pipeab.jsonl" 2> "${O}_pipeab.err" || fail pipeab $?
    cut -c1-200 "${O}_pipeab.jsonl" ;;
  alg)
    # FTRL / FTL kernel times on the resident batches (tools/alg_probe.py; ALG_SHORT=1: the
    # few-wave d = 64 ones)
    OCX_PROBE_SHORT=${ALG_SHORT:-} timeout -k 10 400 python -u tools/alg_probe.py > "${O}_alg.jsonl" 2> "${O}_alg.err" || fail alg $?
    cut -c1-200 "${O}_alg.jsonl" ;;
  algsq)
    # SQ counters of the pipelined FTRL and FTL kernels on the few-wave 4 900 x 1e5 x 64 batch
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "${O}_algsq" -o sq -- python3 "$R/tools/alg_sq.py" ${ALGSQ_SHAPE:-4900 100000 64} > "${O}_algsq.log" 2>&1) || fail algsq $?
    python tools/pmc_summary.py --kernel alg_pipe "${O}_algsq" ;;
  overlap)
    timeout -k 10 400 python -u tools/overlap_probe.py > "${O}_overlap.jsonl" 2> "${O}_overlap.err" || fail overlap $?
    cut -c1-260 "${O}_overlap.jsonl" ;;
  pipetraffic)
    # HBM bytes of the overlapped pipeline's kernels (two PMC passes over two batches; the
    # counters serialise the dispatches, so these runs are for bytes, not time)
    for C in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export TMPDIR=/tmp && OCX_PROBE_NB=2 OCX_PROBE_SEQ=0 OCX_PROBE_CONFIGS=4:0:2:2 timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "${O}_ppmc_$C" -o pmc -- python3 "$R/tools/overlap_probe.py" > "${O}_ppmc_$C.log" 2>&1) || fail "pipe pmc $C" $?
    done
    python tools/pipe_traffic.py "${O}_ppmc_FETCH_SIZE" "${O}_ppmc_WRITE_SIZE" > "${O}_pipetraffic.json" || fail pipetraffic $?
    cat "${O}_pipetraffic.json" ;;
  overlaptrace)
    (cd /tmp && export TMPDIR=/tmp && OCX_PROBE_NB=4 OCX_PROBE_CONFIGS=${OTRACE_CONFIG:-4:0:2:2} timeout -k 10 400 rocprofv3 --kernel-trace -d "${O}_otrace" -o ot --output-format csv -- python3 "$R/tools/overlap_probe.py" > "${O}_otrace.log" 2>&1) || fail overlaptrace $?
    python tools/overlap_report.py "${O}_otrace" > "${O}_otrace.json" || fail overlap_report $?
    cut -c1-400 "${O}_otrace.json" ;;
  trail)
    timeout -k 10 600 python -u tools/trail_probe.py --cases "${TRAIL_CASES:-c4,t1e5}" --chunks "${TRAIL_CHUNKS:-12}" --ramps "${TRAIL_RAMPS:-}" > "${O}_trail.jsonl" 2> "${O}_trail.err" || fail trail $?
    cut -c1-260 "${O}_trail.jsonl" ;;
  trailtrace)
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "${O}_ttrace" -o tt --output-format csv -- python3 "$R/tools/trail_probe.py" --cases t1e5 --runs-t5 19600 --check 0 > "${O}_ttrace.log" 2>&1) || fail trailtrace $?
    ls "${O}_ttrace" ;;
  trailtraffic)
    # HBM bytes of the trailing pipeline on two T = 1e5 batches (9 800 runs), two PMC passes
    for C in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "${O}_tpmc_$C" -o pmc -- python3 "$R/tools/trail_probe.py" --cases t1e5 --runs-t5 9800 --only-trailing --check 0 > "${O}_tpmc_$C.log" 2>&1) || fail "trail pmc $C" $?
    done
    python tools/trail_traffic.py "${O}_tpmc_FETCH_SIZE" "${O}_tpmc_WRITE_SIZE" 9800 100000 > "${O}_trailtraffic.json" || fail trailtraffic $?
    cat "${O}_trailtraffic.json" ;;
  genwaves)
    timeout -k 10 300 python -u tools/genwaves_probe.py > "${O}_genwaves.jsonl" 2> "${O}_genwaves.err" || fail genwaves $?
    cat "${O}_genwaves.jsonl"
    i=0
    for CS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
              "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC" \
              "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64"; do
      i=$((i + 1))
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $CS --output-format csv -d "${O}_gwpmc$i" -o pmc -- python3 "$R/tools/genwaves_probe.py" --reps 1 > "${O}_gwpmc$i.log" 2>&1) || fail "genwaves pmc $i" $?
    done
    python tools/pmc_summary.py "${O}_gwpmc1" "${O}_gwpmc2" "${O}_gwpmc3" --kernel ocx_gen_wave --by-grid > "${O}_genwaves_pmc.txt"
    cat "${O}_genwaves_pmc.txt" ;;
  config4)
    timeout -k 10 500 python -u tools/config4_probe.py ${C4ARGS:-} > "${O}_config4.jsonl" 2> "${O}_config4.err" || fail config4 $?
    cat "${O}_config4.jsonl" ;;
  gpusub)
    # a subset of the GPU suite: GPUSUB="-k expr" (or test files) chosen per call
    timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread ${GPUSUB:-tests} > "${O}_gpusub.log" 2>&1
    rc=$?; tail -3 "${O}_gpusub.log"
    [ $rc -eq 0 ] || fail gpusub $rc ;;
  genscale)
    timeout -k 10 300 python -u tools/genscale_probe.py > "${O}_genscale.jsonl" 2> "${O}_genscale.err" || fail genscale $?
    cat "${O}_genscale.jsonl" ;;
  cumask)
    timeout -k 10 60 tools/cumask_map > "${O}_cumask_map.txt" 2>&1 || fail cumask_map $?
    timeout -k 10 240 python -u tools/cumask_probe.py > "${O}_cumask.jsonl" 2> "${O}_cumask.err" || fail cumask $?
    cat "${O}_cumask_map.txt" "${O}_cumask.jsonl" ;;
  layout)
    timeout -k 10 400 python -u tools/e2e_layout.py > "${O}_layout.jsonl" 2> "${O}_layout.err" || fail layout $?
    cut -c1-200 "${O}_layout.jsonl" ;;
  smallpipe)
    timeout -k 10 400 python -u tools/small_pipe_probe.py > "${O}_smallpipe.jsonl" 2> "${O}_smallpipe.err" || fail smallpipe $?
    cut -c1-220 "${O}_smallpipe.jsonl" ;;
  smalld)
    timeout -k 10 400 python -u tools/gt_small_d.py > "${O}_smalld.jsonl" 2> "${O}_smalld.err" || fail smalld $?
    cut -c1-200 "${O}_smalld.jsonl" ;;
  smart)
    timeout -k 10 400 python -u tools/smart_probe.py > "${O}_smart.jsonl" 2> "${O}_smart.err" || fail smart $?
    cut -c1-200 "${O}_smart.jsonl" ;;
  twin)
    timeout -k 10 400 python -u tools/twin32_probe.py > "${O}_twin.jsonl" 2> "${O}_twin.err" || fail twin $?
    cut -c1-200 "${O}_twin.jsonl" ;;
  exact)
    timeout -k 10 400 python -u tools/exact_probe.py > "${O}_exact.jsonl" 2> "${O}_exact.err" || fail exact $?
    cut -c1-200 "${O}_exact.jsonl" ;;
  config3)
    # configs[2]: FTRL vs exact FTL, 1e5 trials x 1e4 x 64, generation included
    timeout -k 10 600 python tools/perf_extra.py config3 > "${O}_config3.log" 2>&1 || fail config3 $?
    grep '^{' "${O}_config3.log" | cut -c1-220 ;;
  sweep)
    timeout -k 10 900 python tools/perf_extra.py sweep config4 > "${O}_sweep.log" 2>&1 || fail sweep $?
    grep '^{' "${O}_sweep.log" | cut -c1-220 ;;
  *) echo "unknown step $step"; exit 64 ;;
  esac
done
