set -o pipefail
# hgemm fp32 epilogues without per-store drains: tests, then GPT-2 same-box A/B vs abso/base_C.so (bench + per-kernel)
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_hgemm_gpu.py tests/test_models_gpu.py tests/test_model_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1 || { tail -30 gpurun_out/r6e_tests.log; exit 1; }
tail -1 gpurun_out/r6e_tests.log
bash scripts/gpu_ab_env.sh gpt2 DPE_EXT_SO=$GRAFT_REPO_ROOT/abso/base_C.so 3 || exit 1
MARK=adam_kernel BENCH_ARGS="--model gpt2" TOP=30 bash scripts/gpu_ab_steady.sh $GRAFT_REPO_ROOT/abso/base_C.so 1 || exit 1
mkdir -p gpurun_out/abs_gpt2 && cp gpurun_out/abs/steady_*.txt gpurun_out/abs_gpt2/
bash scripts/gpu_ab_env.sh resnet50 DPE_EXT_SO=$GRAFT_REPO_ROOT/abso/base_C.so 2
