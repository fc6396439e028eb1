set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6c_tests.log 2>&1 || { tail -30 gpurun_out/r6c_tests.log; exit 1; }
tail -1 gpurun_out/r6c_tests.log
bash scripts/gpu_ab_env.sh gpt2 DPE_EXT_SO=$GRAFT_REPO_ROOT/abso/base_C.so 3
