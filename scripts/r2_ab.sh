set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/ab_hgemm.py --rounds 5 --shapes sq4096.fwd,sq4096.dgrad,sq8192.fwd,sq8192.dgrad,sq8192.wgrad,qkv.fwd,fc.dgrad,lmhead.fwd,lmhead.dgrad,fc.wgrad --arm rowmajor:-1,-1,-1 --arm g4:-1,-1,4 --arm g8:-1,-1,8 --arm g16:-1,-1,16 > gpurun_out/ab_group.jsonl 2>&1 || exit 1
