#!/bin/bash
# GPU-box sequence: each step under its own time limit; stop on a fault/abort/timeout
# (134/139/124/137 or signals), continue past ordinary failures (exit 1).
mkdir -p gpurun_out
run() {  # name, seconds, cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "STOP after $name (rc=$rc)"; exit $rc ;; esac
}
export PYTHONUNBUFFERED=1
for step in "$@"; do
  case $step in
    build) run build 300 python -c "import __graft_entry__ as g; g.build()" ;;
    tests) run gpu_tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 600 python bench.py ;;
    bench10) run bench10 600 python bench.py --repeats 10 --no-cpu-baseline ;;
    headline) run headline 300 python bench.py --sections headline --no-cpu-baseline ;;
    repeats2) run repeats2 300 python bench.py --repeats 2 --sections headline --no-cpu-baseline ;;
    # bench.py --gpus 2 launches its own ranks (torch.distributed.run child); gloo rehearsal with
    # both ranks on cuda:0 (the driver's 8-GPU runs use RCCL, one GPU per rank)
    rank2) XPG_BENCH_BACKEND=gloo XPG_BENCH_ONE_GPU=1 run rank2 500 python bench.py --gpus 2 --sections headline,c3 --no-cpu-baseline --steps 20 ;;
    capture) run capture 400 python tools/capture_probe.py ;;
    capbisect) run capture_bisect 400 python tools/capture_probe.py wait_empty wait_chain seq3 pingpong ring3_late ring3_first ring3x2 "p2:g=1,prod=0,fin=0,fit=0,u=1" "p2:g=1,prod=0,fin=0,fit=0,u=2" ;;
    capbisect2) run capture_bisect2 400 python tools/capture_probe.py pingpong_cur pingpong_join_first pingpong_nowork_b pingpong_end ;;
    # headline PMC passes on the grouped pipeline: --steps 6 --warmup 2 = groups of 2: 1 warm-up +
    # 3 eager phase groups + 1 eager dev-seed group + 3 graph groups + 1 graph-check group = 9 ops
    pmc_hl) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run pmc_fetch_headline 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_fetch_headline -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --sections headline && \
           run pmc_write_headline 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_write_headline -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --sections headline ;;
    hl3) for r in 1 2 3; do run hl_$r 200 python bench.py --sections headline,node_c3 --no-cpu-baseline; done ;;
    wlmtests) run wlmtests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coverage.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "wlm or run_queries or graph" ;;
    gfprobe) run gfprobe 120 ./tools/gf_probe 1000000 25600 512 3 && run gfprobe_noload 120 ./tools/gf_probe 1000000 25600 512 3 1 && run gfprobe_ns 120 ./tools/gf_probe_ns 1000000 25600 512 3 ;;
    gfabl) for d in 0 1 2 4; do run gfabl_$d 120 ./tools/gf_probe_abl 1000000 25600 512 2 $d || exit 1; done ;;
    rccl1) run rccl1 400 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v -rf --timeout 360 --timeout-method thread -k rccl_one_rank ;;
    gfl2) run gfl2 120 ./tools/gf_probe 1000000 25600 512 3 8 ;;
    gfg4) run gfg4 120 ./tools/gf_probe_g4 1000000 25600 512 3 && run gfg4_nl 120 ./tools/gf_probe_g4 1000000 25600 512 3 1 ;;
    gfpmc) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run gfpmc1 120 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/gfpmc1 -o run -- ./tools/gf_probe_ns 1000000 25600 512 2 && \
           run gfpmc2 120 timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/gfpmc2 -o run -- ./tools/gf_probe_ns 1000000 25600 512 2 ;;
    samptests) run samptests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coverage.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "shapley or sampler or mask or seed" ;;
    shaptests) run shaptests 400 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "shap or kernel or golden or explainer_run" ;;
    gftests) run gftests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -rf --timeout 300 --timeout-method thread -k "fused or (oracle_large and grid) or (continuation and grid) or many_columns" ;;
    gpsec) for r in 1 2; do run gp_$r 300 python bench.py --sections gp --no-cpu-baseline; done ;;
    early2) run early2 500 python -u tools/ws_ab.py --rows 64 --reps 3 --variants "OVERLAP=0;OVERLAP=0,EARLY2=1;OVERLAP=0;OVERLAP=0,EARLY2=1;OVERLAP=1;OVERLAP=1,EARLY2=1" ;;
    captests) run captests 200 python -u -m pytest tests/test_gpu_capture.py -m gpu -v -rf --timeout 120 --timeout-method thread ;;
    apitrace) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
              run apitrace 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d gpurun_out/apitrace -o run -- python3 tools/api_first_call_probe.py --queries 8,9,10 ;;
    htrace) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
            run htrace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/htrace -o run -- python3 bench.py --sections headline --no-cpu-baseline --steps 20 ;;
    apigc) run apigc 200 python -u tools/api_first_call_probe.py && PROBE_GC_FREEZE=1 run apigc_freeze 200 python -u tools/api_first_call_probe.py ;;
    overlap) run overlap 500 python tools/ws_ab.py --rows 256 --reps 3 --variants "OVERLAP=0;OVERLAP=1;OVERLAP=0;OVERLAP=1" ;;
    rank2c4) XPG_BENCH_BACKEND=gloo XPG_BENCH_ONE_GPU=1 run rank2c4 500 python bench.py --gpus 2 --sections c4 --no-cpu-baseline && run rank1c4 300 python bench.py --sections c4 --no-cpu-baseline && grep -h result_checksum gpurun_out/rank2c4.log gpurun_out/rank1c4.log | python -c "import sys, json; [print(json.loads(l)['n_gpus'], json.loads(l)['regimes']['hetero_c4']['result_checksum'], json.loads(l)['regimes']['hetero_c4']['ms_per_job']) for l in sys.stdin if l.startswith('{')]" ;;
    rank2c5) XPG_BENCH_BACKEND=gloo XPG_BENCH_ONE_GPU=1 run rank2c5 500 python bench.py --gpus 2 --sections c5 --no-cpu-baseline && run rank1c5 300 python bench.py --sections c5 --no-cpu-baseline && grep -h result_checksum gpurun_out/rank2c5.log gpurun_out/rank1c5.log | python -c "import sys, json; [print(json.loads(l)['n_gpus'], json.loads(l)['regimes']['c5_hetero']['result_checksum'], json.loads(l)['regimes']['c5_hetero']['ms_per_job']) for l in sys.stdin if l.startswith('{')]" ;;
    c5info) run c5info 300 python -u tools/c5_plan_info.py ;;
    c5ab) XPG_AGG_ROWS=0 run c5_aggrows0 300 python bench.py --sections c5 --no-cpu-baseline && run c5_aggrows1 300 python bench.py --sections c5 --no-cpu-baseline && grep -h ms_per_job gpurun_out/c5_aggrows0.log gpurun_out/c5_aggrows1.log | python -c "import sys, json; [print(json.loads(l)['regimes']['c5_hetero']['ms_per_job']) for l in sys.stdin if l.startswith('{')]" ;;
    prof_*) sec=${step#prof_}
           cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run prof_$sec 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$sec -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --sections $sec ;;
    # layer-2 ablations (c3 full size, one 32-row pass): full, no MFMA, no gathers, no epilogue,
    # exact f32 (B3=0) beside the default bf16x3
    wsdbg) XPG_DIAGNOSTICS=1 run wsdbg 500 python tools/ws_ab.py --variants "B3=1;B3=1,DBG=16;B3=1,DBG=32;B3=1,DBG=64;B3=0" ;;
    # FETCH_SIZE / WRITE_SIZE factors per access shape (tools/fetch_calib.hip, known bytes)
    calib) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/calib_fetch -o run -- ./tools/fetch_calib && \
           run calib_write 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/calib_write -o run -- ./tools/fetch_calib ;;
    fwdprobe) XPG_LIB=tools/libxpgnn_stamps.so run fwdprobe 300 python tools/fwd_probe.py ;;
    # k_wlm_fit_mc mode A/B (tools/wlm_probe stamps, c2 fit shape): 0 base, 1 late stage,
    # 2 split poll, 3 both; alternating rounds on one box
    modes) for r in 1 2; do for md in 0 1 2 3; do XPG_MC_MODE=$md run probe_mode${md}_r$r 120 ./tools/wlm_probe 1193 12800 256; done; done ;;
    gw2) run gw2 300 ./tools/gw2_probe ;;
    gprobe) run gather_probe 180 ./tools/gather_probe ;;
    apitests) run apitests 600 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "explainer or golden or exchange or frame or query or Explainer" ;;
    apisec) run api_sec 300 python bench.py --sections api --no-cpu-baseline ;;
    covtests) run covtests 900 python -u -m pytest tests/test_gpu_coverage.py -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    apirep) run api_repeat 300 python -u tools/api_repeat.py && run api_repeat_nogc 300 python -u tools/api_repeat.py --no-gc && \
            run api_repeat_c3 300 python -u tools/api_repeat.py --graph c3 ;;
    # layer-2 SQ counters (two PMC passes of <= 8 SQ counters) on one c3 pass of ws_ab.py
    wsprof) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run wssq1 300 bash tools/gpu/pmc_pass.sh sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS" "k_wide_l1s|k_wide_last_ws" python3 tools/ws_ab.py --variants "${WSV:-B3=1}" --reps 1 && \
           run wssq2 300 bash tools/gpu/pmc_pass.sh sq2 "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" "k_wide_l1s|k_wide_last_ws" python3 tools/ws_ab.py --variants "${WSV:-B3=1}" --reps 1 ;;
    # c3 HBM counters per kernel (FETCH_SIZE / WRITE_SIZE passes of the c3 bench section)
    c3pmc) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run pmc_fetch_c3 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_fetch_c3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --sections c3 && \
           run pmc_write_c3 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_write_c3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --sections c3 ;;
    apiprof) run apiprof 300 python -u tools/api_profile.py ;;
    # the API section alone, after the headline + c3 sections, and with cProfile of the repeated call
    apictx) run api_alone 300 python bench.py --sections api --no-cpu-baseline && \
            run api_after 400 python bench.py --sections headline,c3,api --no-cpu-baseline && \
            XPG_BENCH_API_PROFILE=1 run api_prof 300 python bench.py --sections headline,c3,api --no-cpu-baseline ;;
    # c3 SQ + GRBM counters (MFMA busy, clock, wave waits) of the default and exact-f32 layer 2
    sqc3) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
          run sq_c3_pass 300 bash tools/gpu/pmc_pass.sh sq_c3 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" "k_wide" python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --sections c3 && \
          python tools/sq_json.py gpurun_out/sq_c3 > gpurun_out/sq_c3.json ;;
    # the tests this round added (wide two-thread / two-stream, workspace order, multi-rank c3)
    newtests) run newtests 600 python -u -m pytest tests/test_gpu_coverage.py tests/test_gpu_multirank.py -m gpu -v -rf --timeout 300 --timeout-method thread -k "two_threads or workspace_ordered or multirank or rehearsal" ;;
    # k_agg_l1_rows ablations on the rows_ab plans (XPG_L1_DBG 1: no keep loads, 2: every source
    # the self row, 4: no output stores, or-ed; outputs invalid) + the kernel stats of the unablated run
    l1abl) for d in 0 1 2 3 4 7; do XPG_DIAGNOSTICS=1 XPG_L1_DBG=$d run l1abl_$d 200 python -u tools/rows_ab.py || exit 1; done && \
           cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run rowsprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rowsprof -o run -- python3 tools/rows_ab.py ;;
    apiprof3) run apiprof3 300 python -u tools/api_profile.py --graph c3 && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
              run apitrace3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/apitrace3 -o run -- python3 tools/api_profile.py --graph c3 --top 5 ;;
    widetests) run widetests 600 python -u -m pytest tests/test_gpu_coverage.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "wide or c3 or hub" ;;
    idxab) run idxab 600 python -u tools/ws_ab.py --variants "${IDXAB:-B3=1,IDX=0;B3=1;B3=1,IDX=0;B3=1;B3=1,RP=6}" ;;
    probe) XPG_WLM=single run probe 120 ./tools/wlm_probe 1193 12800 256 && run probe_mc 120 ./tools/wlm_probe 1193 12800 256 ;;
    profall) cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run profall 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profall -o run -- python3 bench.py --no-cpu-baseline ;;
    benchall) run benchall 900 python bench.py ;;
    prof)  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmc)   cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline && \
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmc_*) # per-section PMC passes: pmc_<section> (headline fits: 1 warmup + 3 eager phase steps + 1 eager
           # dev-seed step + 5 pipelined graph replays + 1 eager graph-check step = 11 ops;
           # c3 / gp: 1 warm-up + 3 timed forwards / repeats = 4 ops)
           sec=${step#pmc_}
           cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
           run pmc_fetch_$sec 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_fetch_$sec -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --sections $sec && \
           run pmc_write_$sec 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc_write_$sec -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --sections $sec ;;
  esac
done
