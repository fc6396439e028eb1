// Shared device helpers for the gfx950 (CDNA4) kernels of this framework.
// Wave = 64 lanes everywhere; vector types sized for 16-byte global/LDS access.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DPE_HOST_DEVICE __host__ __device__ __forceinline__
#define DPE_DEVICE __device__ __forceinline__

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

typedef uint16_t bf16_t;  // storage type for bf16 in global memory

DPE_DEVICE float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN stays NaN: handled by the cast path).
DPE_DEVICE uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // hipcc emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(uint16_t, b);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// One two-source v_cvt_pk_bf16_f32 (RNE, NaN-preserving).  Packing two scalar f2bf() results
// instead costs two converts plus a shift and an or where the compiler does not merge them.
DPE_DEVICE uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{lo, hi}), bf16x2_t));
}

DPE_DEVICE void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

DPE_DEVICE u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack_bf2(f[2 * i], f[2 * i + 1]);
  return r;
}

// ReLU-mask bits of 8 packed bf16 values: bit e = (v[e] > 0), i.e. sign clear and nonzero
DPE_DEVICE uint8_t relu_mask_byte(const u32x4& pk) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lo = pk[j] & 0xffffu, hi = pk[j] >> 16;
    b |= (uint32_t)(lo != 0 && !(lo & 0x8000u)) << (2 * j);
    b |= (uint32_t)(hi != 0 && !(hi & 0x8000u)) << (2 * j + 1);
  }
  return (uint8_t)b;
}

// Barrier for LDS data only: this wave's LDS ops complete, then s_barrier.  __syncthreads() is a
// workgroup-scope release + acquire, which on this target also drains vmcnt(0) -- inside a streaming
// loop that waits for every load / DMA prefetched for later rows or tiles and for the earlier stores.
DPE_DEVICE void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Raw buffer resource over [base, base + bytes): an offset past `bytes` reads zeros / drops the store, so
// a streaming kernel's loads and stores can be issued unconditionally (a load or store under a
// lane-divergent branch makes the compiler's later waits vmcnt(0): the op count differs between paths).
constexpr uint32_t BUF_OOB = 0xfffffff0u;  // past any resource of < 0xffffff00 bytes
DPE_DEVICE __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

DPE_DEVICE float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

DPE_DEVICE float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64).  `sh` >= 16 floats.
DPE_DEVICE float block_sum(float v, float* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = warp_sum(v);
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = (lane < nw) ? sh[lane] : 0.f;
  r = warp_sum(r);
  return r;
}

DPE_DEVICE float block_max(float v, float* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = warp_max(v);
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = (lane < nw) ? sh[lane] : -INFINITY;
  return warp_max(r);
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): blocks b and b+8 share an XCD, so give
// each XCD a contiguous run of logical tiles.
DPE_DEVICE int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

// Philox-4x32-10 counter-based RNG (for dropout masks).
DPE_DEVICE u32x4 philox4x32(uint64_t seed, uint64_t counter_hi, uint32_t counter_lo) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t c0 = counter_lo, c1 = (uint32_t)counter_hi, c2 = (uint32_t)(counter_hi >> 32), c3 = 0x9E3779B9u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  u32x4 r;
  r[0] = c0; r[1] = c1; r[2] = c2; r[3] = c3;
  return r;
}

#define DPE_CHECK_LAUNCH() (void)hipGetLastError()
