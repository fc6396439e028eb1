#!/usr/bin/env python3
"""ResNet-50 (batch 512, 224^2) convolutions of one steady step: compulsory vs measured HBM bytes, achieved
FLOP rate and distance from the roofline.

input: the per-dispatch table of scripts/pmc_dispatch_step.py (gpurun_out/pmcs/resnet50_dispatch.txt; one
steady step of bench.py under two rocprofv3 --pmc passes, dispatch index 0 = the first kernel after the
previous step's SGD kernel).  Every row below names the representative dispatch(es) of one conv role, is
checked against the kernel the table shows there, and counts how many times per step that role runs.

compulsory bytes: every operand tensor read once and the result written once (bf16 NHWC activations,
M x C x 2 B; weights ignored -- <= 9.4 MB); a strided 1x1 conv's input counts only its sampled pixels.
roofline: max(compulsory bytes / 6.0 TB/s -- the rate this step's BN passes sustain, 75 % of the 8 TB/s
datasheet figure --, FLOPs / 2.5 PF dense bf16).  SOL = roofline time / measured time.
Measured times come from the profiled run (counters on: ~3-5 % slower than the plain bench).

usage: sol_table.py <resnet50_dispatch.txt>"""
import re
import sys

BW, PEAK = 6.0e12, 2.5e15
M1, M2, M3, M4 = 512 * 56 * 56, 512 * 28 * 28, 512 * 14 * 14, 512 * 7 * 7


def T(m, c):  # bytes of an [m, c] bf16 activation
    return m * c * 2


def F(m, n, k):  # GEMM FLOPs
    return 2.0 * m * n * k


# (role, dispatch indices summed as one call, calls per step, kernel substring, compulsory read, write, FLOPs)
ROWS = [
    # ---- forward
    ("L1.0 downsample 1x1 64->256", [13], 1, "pw_stream", T(M1, 64), T(M1, 256), F(M1, 256, 64)),
    ("L1.0 conv1 1x1 64->64", [15], 1, "igemm_dma", T(M1, 64), T(M1, 64), F(M1, 64, 64)),
    ("L1 conv2 3x3 64 (BN on load)", [17], 3, "conv3x3_rows", T(M1, 64), T(M1, 64), F(M1, 64, 576)),
    ("L1 conv3 1x1 64->256 + residual", [23], 3, "pw_stream", T(M1, 64) + T(M1, 256), T(M1, 256), F(M1, 256, 64)),
    ("L1.1-2 conv1 1x1 256->64", [24], 2, "igemm_dma", T(M1, 256), T(M1, 64), F(M1, 64, 256)),
    ("L2.0 downsample 1x1/s2 256->512", [42], 1, "igemm_dma", T(M2, 256), T(M2, 512), F(M2, 512, 256)),
    ("L2.0 conv1 1x1 256->128 @56", [44], 1, "igemm_dma", T(M1, 256), T(M1, 128), F(M1, 128, 256)),
    ("L2.0 conv2 3x3/s2 128", [47], 1, "igemm_dma", T(M1, 128), T(M2, 128), F(M2, 128, 1152)),
    ("L2 conv3 1x1 128->512 + residual", [53], 4, "pw_stream", T(M2, 128) + T(M2, 512), T(M2, 512), F(M2, 512, 128)),
    ("L2.1-3 conv1 1x1 512->128", [54], 3, "igemm_dma", T(M2, 512), T(M2, 128), F(M2, 128, 512)),
    ("L2.1-3 conv2 3x3 128", [57], 3, "igemm_dma", T(M2, 128), T(M2, 128), F(M2, 128, 1152)),
    ("L3.0 downsample 1x1/s2 512->1024", [84], 1, "hgemm", T(M3, 512), T(M3, 1024), F(M3, 1024, 512)),
    ("L3.0 conv1 1x1 512->256 @28", [86], 1, "igemm_dma", T(M2, 512), T(M2, 256), F(M2, 256, 512)),
    ("L3.0 conv2 3x3/s2 256", [89], 1, "hgemm", T(M2, 256), T(M3, 256), F(M3, 256, 2304)),
    ("L3 conv3 1x1 256->1024 + residual", [96], 5, "pw_stream", T(M3, 256) + T(M3, 1024), T(M3, 1024), F(M3, 1024, 256)),
    ("L3.1-5 conv1 1x1 1024->256", [97], 5, "hgemm", T(M3, 1024), T(M3, 256), F(M3, 256, 1024)),
    ("L3.1-5 conv2 3x3 256", [100], 5, "hgemm", T(M3, 256), T(M3, 256), F(M3, 256, 2304)),
    ("L3.5 conv3 1x1 256->1024 (stats)", [147], 1, "pw_stream", T(M3, 256), T(M3, 1024), F(M3, 1024, 256)),
    ("L4.0 downsample 1x1/s2 1024->2048", [150], 1, "hgemm", T(M4, 1024), T(M4, 2048), F(M4, 2048, 1024)),
    ("L4.0 conv1 1x1 1024->512 @14", [152], 1, "hgemm", T(M3, 1024), T(M3, 512), F(M3, 512, 1024)),
    ("L4.0 conv2 3x3/s2 512", [155], 1, "hgemm", T(M3, 512), T(M4, 512), F(M4, 512, 4608)),
    ("L4 conv3 1x1 512->2048", [158], 3, "igemm_dma", T(M4, 512), T(M4, 2048), F(M4, 2048, 512)),
    ("L4.1-2 conv1 1x1 2048->512", [161], 2, "hgemm", T(M4, 2048), T(M4, 512), F(M4, 512, 2048)),
    ("L4.1-2 conv2 3x3 512", [164], 2, "hgemm", T(M4, 512), T(M4, 512), F(M4, 512, 4608)),
    # ---- backward, layer 4 (wgrad: dW = x^T dz, split-K partials + finalize not counted; dgrad + BNB: the
    # data grad with the next BN-backward's partials from the pre-BN input h in the epilogue)
    ("L4 wgrad conv3", [194], 3, "hgemm", T(M4, 2048) + T(M4, 512), 0, F(M4, 2048, 512)),
    ("L4 dgrad conv3 + BNB", [196], 3, "hgemm", T(M4, 2048) + T(M4, 512), T(M4, 512), F(M4, 512, 2048)),
    ("L4.1-2 wgrad conv2 3x3", [199], 2, "hgemm", 2 * T(M4, 512), 0, F(M4, 512, 4608)),
    ("L4.1-2 dgrad conv2 3x3 + BNB", [202], 2, "hgemm", 2 * T(M4, 512), T(M4, 512), F(M4, 512, 4608)),
    ("L4.1-2 wgrad conv1", [205], 2, "hgemm", T(M4, 512) + T(M4, 2048), 0, F(M4, 512, 2048)),
    ("L4.1-2 dgrad conv1 + residual", [207], 2, "igemm_dma", T(M4, 512) + T(M4, 2048), T(M4, 2048), F(M4, 2048, 512)),
    ("L4.0 wgrad conv2 3x3/s2", [232], 1, "hgemm", T(M4, 512) + T(M3, 512), 0, F(M4, 512, 4608)),
    ("L4.0 dgrad conv2 3x3/s2 + BNB (4 phases)", [234, 235, 236, 237], 1, "igemm_dma", T(M4, 512) + T(M3, 512), T(M3, 512), F(M4, 512, 4608)),
    ("L4.0 wgrad conv1 @14", [240], 1, "hgemm", T(M3, 512) + T(M3, 1024), 0, F(M3, 512, 1024)),
    ("L4.0 wgrad downsample", [242], 1, "hgemm", T(M4, 2048) + T(M4, 1024), 0, F(M4, 2048, 1024)),
    ("L4.0 dgrad conv1 @14", [244], 1, "igemm_dma", T(M3, 512), T(M3, 1024), F(M3, 1024, 512)),
    ("L4.0 dgrad downsample (strided, accumulate)", [245], 1, "igemm_dma", T(M4, 2048) + T(M4, 1024), T(M4, 1024), F(M4, 1024, 2048)),
    # ---- layer 3
    ("L3 wgrad conv3", [249], 6, "hgemm", T(M3, 1024) + T(M3, 256), 0, F(M3, 1024, 256)),
    ("L3.5 dgrad conv3 + BNB", [251], 1, "hgemm", T(M3, 1024) + T(M3, 256), T(M3, 256), F(M3, 256, 1024)),
    ("L3.0-4 dgrad conv3 (Gram BN3-bwd on A) + BNB", [267], 5, "hgemm", T(M3, 1024) + T(M3, 256), T(M3, 256), F(M3, 256, 1024)),
    ("L3.1-5 wgrad conv2 3x3", [254], 5, "hgemm", 2 * T(M3, 256), 0, F(M3, 256, 2304)),
    ("L3.1-5 dgrad conv2 3x3 + BNB", [256], 5, "hgemm", 2 * T(M3, 256), T(M3, 256), F(M3, 256, 2304)),
    ("L3.1-5 wgrad conv1", [259], 5, "hgemm", T(M3, 256) + T(M3, 1024), 0, F(M3, 256, 1024)),
    ("L3.2-5 dgrad conv1 + residual", [261], 4, "pw_stream", T(M3, 256) + T(M3, 1024), T(M3, 1024), F(M3, 1024, 256)),
    ("L3.0 wgrad conv2 3x3/s2", [336], 1, "hgemm", T(M3, 256) + T(M2, 256), 0, F(M3, 256, 2304)),
    ("L3.0 dgrad conv2 3x3/s2 + BNB (4 phases)", [338, 339, 340, 341], 1, "igemm_dma", T(M3, 256) + T(M2, 256), T(M2, 256), F(M3, 256, 2304)),
    ("L3.0 wgrad conv1 @28", [344], 1, "hgemm", T(M2, 256) + T(M2, 512), 0, F(M2, 256, 512)),
    ("L3.0 wgrad downsample", [346], 1, "hgemm", T(M3, 1024) + T(M3, 512), 0, F(M3, 1024, 512)),
    ("L3.0 dgrad conv1 @28 + downsample dX", [349], 1, "pw_stream", T(M2, 256) + T(M3, 512), T(M2, 512), F(M2, 512, 256)),
    # ---- layer 2
    ("L2 wgrad conv3", [350], 4, "igemm_wgrad", T(M2, 512) + T(M2, 128), 0, F(M2, 512, 128)),
    ("L2 dgrad conv3 (Gram BN3-bwd on A) + BNB", [355], 4, "pw_cat", T(M2, 512) + T(M2, 128), T(M2, 128), F(M2, 128, 512)),
    ("L2.1-3 wgrad conv2 3x3", [358], 3, "igemm_wgrad", 2 * T(M2, 128), 0, F(M2, 128, 1152)),
    ("L2.1-3 dgrad conv2 3x3 + BNB", [359], 3, "igemm_dma", 2 * T(M2, 128), T(M2, 128), F(M2, 128, 1152)),
    ("L2.1-3 wgrad conv1", [362], 3, "igemm_wgrad", T(M2, 128) + T(M2, 512), 0, F(M2, 128, 512)),
    ("L2.2-3 dgrad conv1 + residual", [363], 2, "pw_stream", T(M2, 128) + T(M2, 512), T(M2, 512), F(M2, 512, 128)),
    ("L2.0 wgrad conv2 3x3/s2", [402], 1, "igemm_wgrad", T(M2, 128) + T(M1, 128), 0, F(M2, 128, 1152)),
    ("L2.0 dgrad conv2 3x3/s2 + BNB (4 phases)", [403, 404, 405, 406], 1, "igemm_dma", T(M2, 128) + T(M1, 128), T(M1, 128), F(M2, 128, 1152)),
    ("L2.0 wgrad conv1 @56", [409], 1, "igemm_wgrad", T(M1, 128) + T(M1, 256), 0, F(M1, 128, 256)),
    ("L2.0 wgrad downsample", [410], 1, "hgemm", T(M2, 512) + T(M2, 256), 0, F(M2, 512, 256)),
    ("L2.0 dgrad downsample (strided)", [412], 1, "igemm_dma", T(M2, 512), T(M2, 256), F(M2, 256, 512)),
    ("L2.0 dgrad conv1 @56 + downsample dX", [413], 1, "pw_stream", T(M1, 128) + T(M2, 256), T(M1, 256), F(M1, 256, 128)),
    # ---- layer 1
    ("L1 wgrad conv3", [414], 3, "igemm_wgrad", T(M1, 256) + T(M1, 64), 0, F(M1, 256, 64)),
    ("L1 dgrad conv3 (Gram BN3-bwd on A) + BNB", [419], 3, "pw_cat", T(M1, 256) + T(M1, 64), T(M1, 64), F(M1, 64, 256)),
    ("L1 wgrad conv2 3x3", [422], 3, "wgrad3x3_rows", 2 * T(M1, 64), 0, F(M1, 64, 576)),
    ("L1 dgrad conv2 3x3 + BNB", [425], 3, "conv3x3_rows", 2 * T(M1, 64), T(M1, 64), F(M1, 64, 576)),
    ("L1.1-2 wgrad conv1", [428], 2, "igemm_wgrad", T(M1, 64) + T(M1, 256), 0, F(M1, 64, 256)),
    ("L1.2 dgrad conv1 + residual", [429], 1, "pw_stream", T(M1, 64) + T(M1, 256), T(M1, 256), F(M1, 256, 64)),
    ("L1.0 wgrad conv1", [462], 1, "igemm_wgrad", 2 * T(M1, 64), 0, F(M1, 64, 64)),
    ("L1.0 wgrad downsample", [463], 1, "igemm_wgrad", T(M1, 256) + T(M1, 64), 0, F(M1, 256, 64)),
    ("L1.0 dgrad conv1", [464], 1, "igemm_dma", T(M1, 64), T(M1, 64), F(M1, 64, 64)),
    ("L1.0 dgrad downsample (accumulate)", [465], 1, "igemm_dma", T(M1, 256) + T(M1, 64), T(M1, 64), F(M1, 64, 256)),
    # ---- stem (s2d 4x4x16 input, 112^2 x 64 output; the weight grad recomputes dY from the pooled grad)
    ("stem conv 7x7/s2 (s2d) + stats", [9], 1, "stem_conv", T(M1 * 4, 16), T(M1 * 4, 64), F(M1 * 4, 64, 256)),
    ("stem wgrad (BN + max-pool bwd fused)", [469], 1, "stem_wgrad", T(M1 * 4, 64) + T(M1, 64) + M1 * 64 + T(M1 * 4, 16), 0, F(M1 * 4, 64, 256)),
]


def load(path):
    rows = {}
    for line in open(path):
        m = re.match(r"\s*(\d+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+[\d.]+\s+\d+\s+(.*)", line)
        if m:
            rows[int(m.group(1))] = (float(m.group(2)), float(m.group(3)), float(m.group(4)), float(m.group(5)), m.group(6))
    return rows


def main():
    d = load(sys.argv[1])
    print(f"{'role':46s} {'n':>2} {'us':>7} {'TF/s':>6} {'MFMA%':>5} {'rd MB':>7} {'comp':>7} {'x':>5} "
          f"{'wr MB':>6} {'comp':>6} {'TB/s':>5} {'roof':>6} {'SOL%':>5}  kernel")
    tot = tot_roof = 0.0
    worst = []
    for role, idx, n, kname, rd_c, wr_c, fl in ROWS:
        got = [d.get(i) for i in idx]
        if any(g is None or kname not in g[4] for g in got):
            print(f"{role:46s}  (dispatch {idx} is not a {kname} kernel in this table: re-map)")
            continue
        us = sum(g[0] for g in got)
        mf = sum(g[0] * g[1] for g in got) / us
        rd, wr = sum(g[2] for g in got), sum(g[3] for g in got)
        roof = max((rd_c + wr_c) / BW, fl / PEAK) * 1e6
        tot += n * us
        tot_roof += n * roof
        worst.append((n * (us - roof), role))
        short = re.sub(r"void dpe::|dpe::", "", got[0][4])[:44]
        print(f"{role:46s} {n:2d} {us:7.1f} {fl / us / 1e6:6.0f} {mf:5.1f} {rd:7.0f} {rd_c / 1e6:7.0f} {rd / (rd_c / 1e6):5.2f} "
              f"{wr:6.0f} {wr_c / 1e6:6.0f} {(rd + wr) / us:5.2f} {roof:6.1f} {100 * roof / us:5.0f}  {short}")
    print(f"\nconv total {tot / 1e3:.2f} ms/step (profiled), roofline {tot_roof / 1e3:.2f} ms -> {100 * tot_roof / tot:.0f} % of SOL")
    print("largest gaps (calls x (measured - roofline)):")
    for gap, role in sorted(worst, reverse=True)[:10]:
        print(f"  {gap / 1e3:6.3f} ms  {role}")


if __name__ == "__main__":
    main()
