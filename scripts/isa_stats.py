#!/usr/bin/env python3
"""Per-kernel instruction counts and resource usage from a hipcc --save-temps .s file.
usage: isa_stats.py file.s substring [substring ...]"""
import re, sys

path, names = sys.argv[1], sys.argv[2:]
text = open(path).read()
OPS = ["v_mfma", "v_exp_f32", "ds_read_b128", "ds_read_b64_tr", "ds_write_b128", "ds_bpermute", "v_permlane",
       "s_barrier", "v_max3", "v_max_f32", "v_fma_f32", "v_mul_f32", "v_pk_mul_f32", "v_add_f32", "v_cndmask",
       "v_cvt_pk_bf16", "global_load", "global_store", "buffer_load", "scratch_", "s_waitcnt", "s_cbranch"]
for n in names:
    m = re.search(r"^(_Z\S*" + re.escape(n) + r"\S*):", text, re.M)
    if not m:
        print(n, "not found"); continue
    sym = m.group(1)
    body = text[m.end():text.index(".end_amdhsa_kernel", m.end())]
    print(f"== {sym}")
    meta = {k: re.search(r"\." + k + r"\s+(\d+)", body) for k in
            ["amdhsa_next_free_vgpr", "amdhsa_accum_offset", "amdhsa_next_free_sgpr", "amdhsa_group_segment_fixed_size",
             "amdhsa_private_segment_fixed_size"]}
    print("  " + "  ".join(f"{k.replace('amdhsa_', '')}={v.group(1)}" for k, v in meta.items() if v))
    cnt = {op: len(re.findall(r"^\s+" + op, body, re.M)) for op in OPS}
    print("  " + "  ".join(f"{op}={c}" for op, c in cnt.items()))
