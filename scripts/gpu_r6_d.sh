set -o pipefail
# strided 3x3 data grads (batched remapped epilogue), no-scratch epilogues, LN backward rows: default build vs abso/base_C.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_model_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1 || { tail -30 gpurun_out/r6d_tests.log; exit 1; }
tail -1 gpurun_out/r6d_tests.log
for r in 1 2; do
  echo "new:"; timeout -k 10 200 python scripts/bench_dgrad_bnb.py || exit 1
  echo "base:"; DPE_EXT_SO=$GRAFT_REPO_ROOT/abso/base_C.so timeout -k 10 200 python scripts/bench_dgrad_bnb.py || exit 1
done
bash scripts/gpu_ab_env.sh resnet50 DPE_EXT_SO=$GRAFT_REPO_ROOT/abso/base_C.so 3 || exit 1
MARK=adam_kernel BENCH_ARGS="--model gpt2" TOP=30 bash scripts/gpu_ab_steady.sh $GRAFT_REPO_ROOT/abso/base_C.so 1 || exit 1
mkdir -p gpurun_out/abs_gpt2 && cp gpurun_out/abs/steady_*.txt gpurun_out/abs_gpt2/
MARK=sgd_kernel TOP=60 bash scripts/gpu_ab_steady.sh $GRAFT_REPO_ROOT/abso/base_C.so 1
