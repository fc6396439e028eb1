# Round-3 GPU check: the new / changed GPU tests, then alternating A/B benches of the round's
# switches, the RCCL footprint, the two-launch GEMM decompositions and the CU-budget hog probe.
mkdir -p gpurun_out
timeout -k 10 120 python scripts/debug_bg.py > gpurun_out/r3_debug_bg.txt 2>&1; cut -c1-200 gpurun_out/r3_debug_bg.txt | tail -14
timeout -k 10 600 python -u -m pytest tests/test_hgemm_gpu.py tests/test_model_parity_gpu.py tests/test_ddp_rccl_world2_gpu.py "tests/test_kernels_gpu.py::test_linear_padded_out_features_fwd_bwd" tests/test_models_gpu.py -v -s --timeout 150 --timeout-method thread > gpurun_out/r3_new_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|rel dev|^  [0-9 ]+\|| final weights|survivor|ok: world|ResNet-50 losses" gpurun_out/r3_new_tests.log | cut -c1-250 | tail -90
case $rc in 124|134|137|139) echo "STOP rc=$rc"; exit $rc;; esac
ARMS="- DPE_HGEMM_PLAN2=0" MODEL=gpt2 ROUNDS=2 bash scripts/ab_bench.sh || exit 1
timeout -k 10 300 python scripts/bench_gemm_parts.py > gpurun_out/r3_gemm_parts.jsonl 2>&1; tail -12 gpurun_out/r3_gemm_parts.jsonl
bash scripts/rccl_footprint.sh > gpurun_out/r3_fp.txt 2>&1; tail -4 gpurun_out/r3_fp.txt
