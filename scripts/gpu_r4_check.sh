#!/bin/bash
# Round-4 checks: the new tests first (grouped weight grads, world-4 RCCL incl. rank death, foreign
# writer on fresh grads, step-0 gradient parity), a GPT-2 A/B of the grouped weight grads, then the
# whole GPU suite, smoke and the ResNet bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/r4
timeout -k 10 120 python -u -m pytest -x -v --timeout 100 --timeout-method thread -p no:cacheprovider \
  tests/test_hgemm_gpu.py::test_linear_wgrad_group > gpurun_out/r4/group_test.log 2>&1 || { echo "GROUP TEST FAILED"; tail -40 gpurun_out/r4/group_test.log; exit 1; }
for arm in 0 2 0 2; do
  DPE_GPT2_WGRAD_GROUP=$arm timeout -k 10 200 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/r4/gpt2_g$arm.log 2>&1 || { tail -20 gpurun_out/r4/gpt2_g$arm.log; exit 1; }
  echo "group=$arm $(tail -1 gpurun_out/r4/gpt2_g$arm.log | cut -c1-120)"
done
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_ddp_rccl_world2_gpu.py tests/test_comm_gpu.py::test_gpt2_fresh_gradients_with_foreign_writer \
  tests/test_comm_gpu.py::test_gpt2_fresh_gradients_equal_zeroed \
  "tests/test_model_parity_gpu.py::test_resnet50_step0_gradient_parity" \
  "tests/test_model_parity_gpu.py::test_gpt2_small_step0_gradient_parity_T1024" \
  > gpurun_out/r4/new_tests.log 2>&1 || { echo "NEW TESTS FAILED"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r4/new_tests.log | head -30; tail -40 gpurun_out/r4/new_tests.log; exit 1; }
grep -E "PASSED|FAILED|ok:|survivors|worst|% of bound" gpurun_out/r4/new_tests.log | cut -c1-160
[ "${SKIP_SUITE:-0}" = "1" ] || timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r4/pytest.log 2>&1 || { echo "SUITE FAILED"; tail -40 gpurun_out/r4/pytest.log; exit 1; }
tail -2 gpurun_out/r4/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 || { tail -20 gpurun_out/r4/smoke.log; exit 1; }
tail -1 gpurun_out/r4/smoke.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet.log 2>&1 || { tail -20 gpurun_out/r4/bench_resnet.log; exit 1; }
tail -1 gpurun_out/r4/bench_resnet.log | cut -c1-200
