#!/bin/bash
# Round-6 GPU evidence, in parts that each fit one gpurun call (tools/gpu_steps.sh: every step under its own limit,
# stop at the first fault / time limit).
#   bash tools/r6_gpu.sh tests | full | bench | pmc
# Phases order / io / fe / seg ran experiments whose code was removed after measuring (DESIGN.md §7 rows r6g and
# 'Measured and rejected in round 6'); their env switches no longer exist, so they now time the default build.
case "$1" in
  tests) bash tools/gpu_steps.sh \
    "900 r6_gputests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
    "120 r6_smoke python -c 'import __graft_entry__ as g; g.smoke()'" ;;
  full) bash tools/gpu_steps.sh \
    "400 r6_full_plain python tools/full_size_steps.py --configs c5,c4 --graph" \
    "400 r6_full_coll python tools/full_size_steps.py --configs c5,c4 --graph --train-loop --collectives" ;;
  bench) bash tools/gpu_steps.sh \
    "400 r6_bench python bench.py" ;;
  quick) bash tools/gpu_steps.sh \
    "600 r6_qtests python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_c5_fp16.py tests/test_bench_parity.py tests/test_hip_layers.py -k 'oracle or tie_band or ill_conditioned or consumer_dgrad'" ;;
  fix) bash tools/gpu_steps.sh \
    "700 r6_fixtests python -u -m pytest -q --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_c5_fp16.py tests/test_bench_ddp.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py tests/test_hip_layers.py tests/test_augment.py -k 'c5 or bench_two or distributed_train or rccl or world or upsampler or ill_conditioned or train_loop'" ;;
  study) bash tools/gpu_steps.sh \
    "400 r6_pmc_layers bash tools/r6_pmc_layers.sh" \
    "400 r6_split_ab env SSSEG_TUNE_LOG=1 python tools/split_ab.py" \
    "200 r6_gemm_ceiling python tools/gemm_ceiling.py" ;;
  probe) bash tools/gpu_steps.sh \
    "300 r6_c5 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_c5_fp16.py" \
    "400 r6_bench2 python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_btrace env SSSEG_OVERLAP_TEACHER=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_btrace -o b -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-fp32 --no-graph" ;;
  diag) bash tools/gpu_steps.sh \
    "400 r6_diag_c5v python tools/diag_c5.py full noadv sup" \
    "300 r6_gtrace rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_gtrace -o g -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32" ;;
  wred) bash tools/gpu_steps.sh \
    "600 r6_wred_tests python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_overlap.py tests/test_graph.py tests/test_determinism.py tests/test_c5_fp16.py tests/test_trainer_gpu.py" \
    "200 r6_wred_b1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_wred_b0 env SSSEG_WGRAD_BATCH_REDUCE=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_wred_b1b python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_wred_b0b env SSSEG_WGRAD_BATCH_REDUCE=0 python bench.py --no-cpu-baseline --no-fp32" ;;
  stem) bash tools/gpu_steps.sh \
    "300 r6_c5b python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_c5_fp16.py tests/test_overlap.py" \
    "200 r6_stem1 python tools/bench_stem.py" \
    "200 r6_stem0 env SSSEG_STEM=0 SSSEG_TUNE_LOG=1 python tools/bench_stem.py" \
    "200 r6_stem_b1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_stem_b0 env SSSEG_STEM=0 python bench.py --no-cpu-baseline --no-fp32" ;;
  pmc) bash tools/gpu_steps.sh \
    "300 r6_layers python tools/layer_report.py" \
    "700 r6_pmc bash tools/pmc_run.sh" ;;
  full3) bash tools/gpu_steps.sh \
    "500 r6_full_c3 python tools/full_size_steps.py --configs c3 --graph --train-loop --collectives" \
    "300 r6_full_c5plain python tools/full_size_steps.py --configs c5 --graph --train-loop" ;;
  events) bash tools/gpu_steps.sh \
    "200 r6_ev_tests python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_probe_events.py" \
    "300 r6_ev_free python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_ev_fenced env SSSEG_PROBE_FENCED=1 python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_ev_trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_ev_trace -o b -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32" ;;
  order) bash tools/gpu_steps.sh \
    "200 r6_ord_b1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_ord_b0 env SSSEG_SUP_BWD_FIRST=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_ord_b1b python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_ord_b0b env SSSEG_SUP_BWD_FIRST=0 python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_ord_trace rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_ord_trace -o b -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32" \
    "700 r6_ord_tests python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_overlap.py tests/test_graph.py tests/test_determinism.py tests/test_c5_fp16.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py" ;;
  gq) bash tools/gpu_steps.sh \
    "200 r6_gq_pc0 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gq_pc0o env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 SSSEG_SUP_BWD_FIRST=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gq_q1 env DEBUG_HIP_FORCE_GRAPH_QUEUES=1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gq_q8 env DEBUG_HIP_FORCE_GRAPH_QUEUES=8 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gq_bs env DEBUG_HIP_GRAPH_BATCH_SIZE=1024 python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_gq_trace env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_gq_trace -o b -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32" ;;
  gb) bash tools/gpu_steps.sh \
    "200 r6_gb_1 env DEBUG_HIP_GRAPH_BATCH_SIZE=1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gb_8 env DEBUG_HIP_GRAPH_BATCH_SIZE=8 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gb_32 env DEBUG_HIP_GRAPH_BATCH_SIZE=32 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gb_128 env DEBUG_HIP_GRAPH_BATCH_SIZE=128 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_gb_def python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_gb_trace env DEBUG_HIP_GRAPH_BATCH_SIZE=8 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_gb_trace -o b -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32" ;;
  io) bash tools/gpu_steps.sh \
    "200 r6_io_2 env SSSEG_ISSUE_ORDER=2 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_io_0 env SSSEG_ISSUE_ORDER=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_io_1 env SSSEG_ISSUE_ORDER=1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_io_mb env DEBUG_CLR_MAX_BATCH_SIZE=4096 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_io_cs env DEBUG_CLR_BATCH_CPU_SYNC_SIZE=4096 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_io_cb env GPU_MAX_COMMAND_BUFFERS=4096 python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_io_trace env SSSEG_ISSUE_ORDER=2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_io_trace -o b -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32" ;;
  fe) bash tools/gpu_steps.sh \
    "200 r6_fe_1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_fe_0 env SSSEG_FORK_EVENT=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_fe_1o0 env SSSEG_ISSUE_ORDER=0 python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_fe_trace rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_fe_trace -o b -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32" ;;
  seg) bash tools/gpu_steps.sh \
    "300 r6_seg_tests python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_graph.py tests/test_overlap.py" \
    "200 r6_seg_1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_seg_0 env SSSEG_GRAPH_SEGMENTS=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_seg_1b python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_seg_0b env SSSEG_GRAPH_SEGMENTS=0 python bench.py --no-cpu-baseline --no-fp32" \
    "300 r6_seg_trace rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_seg_trace -o b -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32" ;;
  mw) bash tools/gpu_steps.sh \
    "200 r6_mw_0 env SSSEG_MERGE_WGRAD=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_mw_1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_mw_0b env SSSEG_MERGE_WGRAD=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_mw_1b python bench.py --no-cpu-baseline --no-fp32" \
    "600 r6_mw_tests env SSSEG_MERGE_WGRAD=0 python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_graph.py tests/test_overlap.py tests/test_determinism.py" ;;
  wred4) bash tools/gpu_steps.sh \
    "400 r6_wred4_1 env SSSEG_WGRAD_BATCH_REDUCE=1 python tools/full_size_steps.py --configs c4,c5 --graph" \
    "400 r6_wred4_0 python tools/full_size_steps.py --configs c4,c5 --graph" ;;
  burst) bash tools/gpu_steps.sh \
    "600 r6_burst_tests env SSSEG_WGRAD_BURST=2 python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_graph.py tests/test_overlap.py tests/test_determinism.py" \
    "200 r6_burst_2 env SSSEG_WGRAD_BURST=2 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_burst_1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_burst_3 env SSSEG_WGRAD_BURST=3 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_burst_2b env SSSEG_WGRAD_BURST=2 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_burst_1b python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_burst_3b env SSSEG_WGRAD_BURST=3 python bench.py --no-cpu-baseline --no-fp32" ;;
  knobs) bash tools/gpu_steps.sh \
    "200 r6_kn_base python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_kn_kernarg env HIP_FORCE_DEV_KERNARG=1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_kn_reps env SSSEG_TUNE_REPS=12 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_kn_w75 env SSSEG_KNOBS=10=75 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_kn_w150 env SSSEG_KNOBS=10=150 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_kn_base2 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_kn_kernarg2 env HIP_FORCE_DEV_KERNARG=0 python bench.py --no-cpu-baseline --no-fp32" ;;
  reps) bash tools/gpu_steps.sh \
    "200 r6_rp_12 env SSSEG_TUNE_REPS=12 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_rp_5 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_rp_24 env SSSEG_TUNE_REPS=24 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_rp_12b env SSSEG_TUNE_REPS=12 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_rp_5b python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_rp_24b env SSSEG_TUNE_REPS=24 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_rp_5c python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_rp_12c env SSSEG_TUNE_REPS=12 python bench.py --no-cpu-baseline --no-fp32" ;;
  knobs2) bash tools/gpu_steps.sh \
    "200 r6_k2_base python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_k2_k14off env SSSEG_KNOBS=14=-1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_k2_k16 env SSSEG_KNOBS=16=-1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_k2_k15 env SSSEG_KNOBS=15=-1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_k2_cbwd0 env SSSEG_OVERLAP_CONSISTENCY_BWD=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_k2_gstat0 env SSSEG_BN_GSTAT=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_k2_base2 python bench.py --no-cpu-baseline --no-fp32" ;;
  cbwd) bash tools/gpu_steps.sh \
    "200 r6_cb_0a env SSSEG_OVERLAP_CONSISTENCY_BWD=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_cb_1a python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_cb_0b env SSSEG_OVERLAP_CONSISTENCY_BWD=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_cb_1b python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_cb_0c env SSSEG_OVERLAP_CONSISTENCY_BWD=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_cb_1c python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_cb_0d env SSSEG_OVERLAP_CONSISTENCY_BWD=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_cb_1d python bench.py --no-cpu-baseline --no-fp32" ;;
  hwq) bash tools/gpu_steps.sh \
    "200 r6_hq_8 env GPU_MAX_HW_QUEUES=8 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_hq_d python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_hq_2 env GPU_MAX_HW_QUEUES=2 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_hq_8b env GPU_MAX_HW_QUEUES=8 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_hq_db python bench.py --no-cpu-baseline --no-fp32" ;;
  ident) bash tools/gpu_steps.sh \
    "200 r6_id_1 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_id_0 env SSSEG_BILINEAR_IDENTITY=0 python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_id_1b python bench.py --no-cpu-baseline --no-fp32" \
    "200 r6_id_0b env SSSEG_BILINEAR_IDENTITY=0 python bench.py --no-cpu-baseline --no-fp32" ;;
  *) echo "usage: $0 tests|full|bench|quick|fix|study|probe|diag|wred|stem|pmc|full3|events|order|gq|gb|io|fe|seg|mw|wred4|burst|knobs|reps|knobs2|cbwd|hwq|ident"; exit 2 ;;
esac
