set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/hog_probe.py 0:256:0 8:256:0 32:256:0 64:256:0 32:512:0 32:256:32768 128:256:0 > gpurun_out/hog.log 2>&1 || { tail -20 gpurun_out/hog.log; exit 1; }
grep hog_blocks gpurun_out/hog.log
