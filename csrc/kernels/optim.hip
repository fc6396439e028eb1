// Fused multi-tensor optimizers: ONE launch updates every parameter of a
// model (replacing the reference's foreach-Adam chain of _foreach_lerp_ /
// mul / addcmul / sqrt / div / add / addcdiv launches).
//
// Each parameter is split into CHUNK-element pieces; the launch grid is the
// list of (tensor, chunk) pairs, prepared once on the host and kept on the
// device.  Per element the kernel reads p, g, state(s) and writes p,
// state(s) and (optionally) the bf16 compute shadow of p that the MFMA
// kernels consume -- so no separate fp32->bf16 cast pass per step.
//
// Hyper-parameters (lr etc.) live in a small device array so a captured
// hipGraph can replay the step while the host edits the learning rate.
#include "common.h"

namespace dpe {

struct TensorDesc {
  float* p;
  const float* g;
  float* s1;        // exp_avg (Adam) / momentum_buffer (SGD)
  float* s2;        // exp_avg_sq (Adam)
  uint16_t* shadow;  // bf16 copy of p (may be null)
  int64_t n;
  int group;
  int step_idx;  // index into steps[] (per-parameter step counters)
};

// Per group, 12 floats: lr, beta1/momentum, beta2/dampening, eps, weight_decay,
// flags(bitfield: 1 nesterov, 2 maximize, 4 decoupled wd), grad_scale, pad...
constexpr int HP = 12;
// 16K elements per block: 256 lanes x 4 (one 16-B access per operand) x 16
// iterations.  Small enough that a 25M-parameter model spreads over ~1.6k
// blocks (>6 per CU, so the streaming loads of several waves overlap), large
// enough that the per-block descriptor fetch is noise.
constexpr int CHUNK = 16384;

// Per-element update rules (shared by the 16-B vector body and the scalar tail).
struct AdamRule {
  float lr, b1, b2, eps, wd, step_size, bc2_sqrt;
  bool maximize, decoupled;
  float gscale;
  DPE_DEVICE AdamRule(const float* h, float step) {
    lr = h[0]; b1 = h[1]; b2 = h[2]; eps = h[3]; wd = h[4];
    const int flags = (int)h[5];
    gscale = h[6];
    maximize = flags & 2; decoupled = flags & 4;
    step_size = lr / (1.f - powf(b1, step));
    bc2_sqrt = sqrtf(1.f - powf(b2, step));
  }
  DPE_DEVICE void operator()(float& p, float g, float& m, float& v) const {
    g *= gscale;
    if (maximize) g = -g;
    if (wd != 0.f) {
      if (decoupled) p *= (1.f - lr * wd);
      else g += wd * p;
    }
    m = m + (1.f - b1) * (g - m);  // lerp, as torch
    v = b2 * v + (1.f - b2) * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p -= step_size * (m / denom);
  }
};

struct SgdRule {
  float lr, mom, damp, wd, gscale;
  bool nesterov, maximize, first;
  DPE_DEVICE SgdRule(const float* h, float step) {
    lr = h[0]; mom = h[1]; damp = h[2]; wd = h[4];
    const int flags = (int)h[5];
    gscale = h[6];
    nesterov = flags & 1; maximize = flags & 2;
    first = step <= 1.f;
  }
  DPE_DEVICE void operator()(float& p, float g, float& b, float&) const {
    g *= gscale;
    if (maximize) g = -g;  // as torch: negate before weight decay and momentum
    if (wd != 0.f) g += wd * p;
    if (mom != 0.f) {
      b = first ? g : mom * b + (1.f - damp) * g;
      g = nesterov ? g + mom * b : b;
    }
    p -= lr * g;
  }
};

// One (tensor, chunk) per block.  When every operand of the tensor is 16-B
// aligned (8-B for the bf16 shadow) -- always the case for parameters and for
// bucket-view gradients of 4-multiple sizes -- each lane moves 4 elements per
// operand per iteration with dwordx4 loads/stores; otherwise (or for the
// ragged tail) one element.  `s2` is only touched by rules that use it.
template <class Rule, bool TWO_STATES>
DPE_DEVICE void optim_chunk(const TensorDesc& d, const Rule& rule, int chunk) {
  const int64_t beg = (int64_t)chunk * CHUNK;
  const int64_t end = min(d.n, beg + CHUNK);
  const bool has_s1 = d.s1 != nullptr;
  const uintptr_t align = (uintptr_t)d.p | (uintptr_t)d.g | (uintptr_t)d.s1 | (TWO_STATES ? (uintptr_t)d.s2 : 0);
  const bool vec = (align & 15) == 0 && ((uintptr_t)d.shadow & 7) == 0;
  int64_t i = beg;
  if (vec) {
    // Software-pipelined one 1024-element step ahead: the next step's loads are issued before this step's
    // stores, so the wait for them counts past those stores (loads and stores share vmcnt: loaded after the
    // stores, every step waited for its predecessor's stores to complete).  Every load and store goes through
    // a buffer resource and is issued unconditionally -- an absent state or shadow is a 0-byte resource
    // (loads read 0, stores are dropped) and the last step's look-ahead re-reads its own elements -- so the
    // compiler's waits stay counted instead of vmcnt(0) (common.h buf_rsrc).
    const int64_t vend = beg + ((end - beg) & ~(int64_t)1023);
    const int nsteps = (int)((vend - beg) >> 10);
    const uint32_t bytes = (uint32_t)((vend - beg) * 4);  // <= 64 KiB (CHUNK)
    const __amdgpu_buffer_rsrc_t prs = buf_rsrc(d.p + beg, bytes), grs = buf_rsrc(d.g + beg, bytes);
    const __amdgpu_buffer_rsrc_t mrs = buf_rsrc(has_s1 ? d.s1 + beg : nullptr, has_s1 ? bytes : 0u);
    const __amdgpu_buffer_rsrc_t vrs = buf_rsrc(TWO_STATES ? d.s2 + beg : nullptr, TWO_STATES ? bytes : 0u);
    const __amdgpu_buffer_rsrc_t srs = buf_rsrc(d.shadow ? d.shadow + beg : nullptr, d.shadow ? bytes / 2 : 0u);
    auto ld = [](__amdgpu_buffer_rsrc_t r, uint32_t o) {
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
    };
    const uint32_t lo = threadIdx.x * 16u;  // the lane's 16 B of a 4-KiB step
    f32x4 pn = ld(prs, lo), gn = ld(grs, lo), mn = ld(mrs, lo), vn = ld(vrs, lo);
    for (int k = 0; k < nsteps; ++k) {
      f32x4 p = pn, m = mn, v = vn;
      const f32x4 g = gn;
      const uint32_t o = lo + (uint32_t)k * 4096u, on = k + 1 < nsteps ? o + 4096u : o;
      pn = ld(prs, on);
      gn = ld(grs, on);
      mn = ld(mrs, on);
      vn = ld(vrs, on);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = p[e], me = m[e], ve = v[e];
        rule(pe, g[e], me, ve);
        p[e] = pe; m[e] = me; v[e] = ve;
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, p), prs, o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, m), mrs, o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), vrs, o, 0, 0);
      u32x2 sh;
      sh[0] = pack_bf2(p[0], p[1]);
      sh[1] = pack_bf2(p[2], p[3]);
      __builtin_amdgcn_raw_buffer_store_b64(sh, srs, o >> 1, 0, 0);
    }
    i = vend;
  }
  for (int64_t j = i + threadIdx.x; j < end; j += 256) {
    float p = d.p[j], m = has_s1 ? d.s1[j] : 0.f, v = TWO_STATES ? d.s2[j] : 0.f;
    rule(p, d.g[j], m, v);
    d.p[j] = p;
    if (has_s1) d.s1[j] = m;
    if (TWO_STATES) d.s2[j] = v;
    if (d.shadow) d.shadow[j] = f2bf(p);
  }
}

__global__ __launch_bounds__(256) void adam_kernel(const TensorDesc* __restrict__ td, const int2* __restrict__ chunks,
                                                   const float* __restrict__ hp, const float* __restrict__ steps) {
  const int2 ck = chunks[blockIdx.x];
  const TensorDesc d = td[ck.x];
  optim_chunk<AdamRule, true>(d, AdamRule(hp + d.group * HP, steps[d.step_idx]), ck.y);
}

__global__ __launch_bounds__(256) void sgd_kernel(const TensorDesc* __restrict__ td, const int2* __restrict__ chunks,
                                                  const float* __restrict__ hp, const float* __restrict__ steps) {
  const int2 ck = chunks[blockIdx.x];
  const TensorDesc d = td[ck.x];
  optim_chunk<SgdRule, false>(d, SgdRule(hp + d.group * HP, steps[d.step_idx]), ck.y);
}

}  // namespace dpe

using namespace dpe;

extern "C" int dpe_optim_chunk_size() { return CHUNK; }
extern "C" int dpe_optim_desc_bytes() { return (int)sizeof(TensorDesc); }

// kind: 0 adam/adamw, 1 sgd
extern "C" int dpe_optim_step(int kind, const void* desc, const void* chunks, int nchunks, const float* hp, const float* steps,
                              hipStream_t st) {
  if (nchunks <= 0) return 0;
  if (kind == 0)
    hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(256), 0, st, (const TensorDesc*)desc, (const int2*)chunks, hp, steps);
  else
    hipLaunchKernelGGL(sgd_kernel, dim3(nchunks), dim3(256), 0, st, (const TensorDesc*)desc, (const int2*)chunks, hp, steps);
  return 0;
}
