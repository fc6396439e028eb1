# hgemm slab finalize with 4 loads in flight: GEMM tests, GPT-2 + ResNet-50 benches, GPT-2 profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "linear or gemm or hgemm or wgrad or gpt2" > gpurun_out/fin_tests.log 2>&1 || { grep -E "FAIL|Error|error|assert" gpurun_out/fin_tests.log | head -30; tail -30 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model gpt2 --steps 30 --warmup 5 > gpurun_out/fg.log 2>&1 || exit 1
  echo "gpt2 $(tail -1 gpurun_out/fg.log | cut -c60-175)"
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/fr.log 2>&1 || exit 1
  echo "r50 $(tail -1 gpurun_out/fr.log | cut -c100-190)"
done
rm -rf gpurun_out/prof_fin
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_fin -o run -- python bench.py --model gpt2 --steps 8 --warmup 3 > gpurun_out/prof_fin.log 2>&1 || exit 1
python scripts/prof_steady.py $(find gpurun_out/prof_fin -name "*.db" | head -1) 2 adam_kernel 30 > gpurun_out/g2_steady_fin.txt
grep -E "wall|finalize|ce_vec" gpurun_out/g2_steady_fin.txt
rm -rf gpurun_out/prof_fin
