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
constexpr int CHUNK = 65536;

__global__ __launch_bounds__(256) void adam_kernel(const TensorDesc* __restrict__ td, const int2* __restrict__ chunks,
                                                   const float* __restrict__ hp, const float* __restrict__ steps) {
  const int2 ck = chunks[blockIdx.x];
  const TensorDesc d = td[ck.x];
  const float* h = hp + d.group * HP;
  const float lr = h[0], b1 = h[1], b2 = h[2], eps = h[3], wd = h[4];
  const int flags = (int)h[5];
  const float gscale = h[6];
  const float step = steps[d.step_idx];
  const float bc1 = 1.f - powf(b1, step);
  const float bc2 = 1.f - powf(b2, step);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const bool maximize = flags & 2, decoupled = flags & 4;
  const int64_t beg = (int64_t)ck.y * CHUNK;
  const int64_t end = min(d.n, beg + CHUNK);
  for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
    float g = d.g[i] * gscale;
    if (maximize) g = -g;
    float p = d.p[i];
    if (wd != 0.f) {
      if (decoupled) p *= (1.f - lr * wd);
      else g += wd * p;
    }
    float m = d.s1[i], v = d.s2[i];
    m = m + (1.f - b1) * (g - m);  // lerp, as torch
    v = b2 * v + (1.f - b2) * g * g;
    d.s1[i] = m;
    d.s2[i] = v;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p -= step_size * (m / denom);
    d.p[i] = p;
    if (d.shadow) d.shadow[i] = f2bf(p);
  }
}

__global__ __launch_bounds__(256) void sgd_kernel(const TensorDesc* __restrict__ td, const int2* __restrict__ chunks,
                                                  const float* __restrict__ hp, const float* __restrict__ steps) {
  const int2 ck = chunks[blockIdx.x];
  const TensorDesc d = td[ck.x];
  const float* h = hp + d.group * HP;
  const float lr = h[0], mom = h[1], damp = h[2], wd = h[4];
  const int flags = (int)h[5];
  const float gscale = h[6];
  const bool nesterov = flags & 1, maximize = flags & 2;
  const bool first = steps[d.step_idx] <= 1.f;
  const int64_t beg = (int64_t)ck.y * CHUNK;
  const int64_t end = min(d.n, beg + CHUNK);
  for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
    float g = d.g[i] * gscale;
    float p = d.p[i];
    if (wd != 0.f) g += wd * p;
    if (mom != 0.f) {
      float b = first ? g : mom * d.s1[i] + (1.f - damp) * g;
      d.s1[i] = b;
      g = nesterov ? g + mom * b : b;
    }
    p = maximize ? p + lr * g : p - lr * g;
    d.p[i] = p;
    if (d.shadow) d.shadow[i] = f2bf(p);
  }
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
