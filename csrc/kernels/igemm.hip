// Implicit-GEMM engine for gfx950: dense GEMM (NT / NN / TN) and NHWC
// convolution forward / data-grad / weight-grad on bf16 MFMA
// (v_mfma_f32_16x16x32_bf16), fp32 accumulate.
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"):
//   * 256 threads = 4 waves in a 2x2 grid; each wave owns a (BM/2)x(BN/2)
//     sub-tile as (BM/32)x(BN/32) 16x16 MFMA tiles.
//   * BK = 32; global -> registers -> LDS staging (register staging because
//     the conv loaders gather / zero-pad), double-buffered LDS, ONE barrier
//     per K-step: next tile's global loads are issued before the MFMAs of the
//     current tile and written to the other buffer after them (T14 split).
//   * K-contiguous operands live in a [rows][32] LDS image read with
//     ds_read_b128 and XOR-swizzled so each 16-lane group of the read hits 16
//     distinct 16-B bank slots (swizzle g = {0,2,3,1} on (row>>2)&3).
//   * M/N-contiguous operands (weight-grad A = dy^T, weight-grad B = im2col x,
//     data-grad B = weights) live in a [32][cols] image read with the CDNA4
//     transposing ds_read_b64_tr_b16 (T10); chunk XOR-swizzle chosen so both
//     32-lane halves of every transposed read are conflict-free.
//   * MFMA operands are issued swapped (D^T = B^T A^T) so each lane ends up
//     holding 4 consecutive output COLUMNS of one output row: the epilogue
//     writes 8-byte packed bf16 to an LDS C tile, then stores whole 16-byte
//     row chunks (coalesced), optionally adding a residual and accumulating
//     per-column sum / sum-of-squares for a following BatchNorm.
//   * Workgroup ids are remapped XCD-aware (bijective) with N-tiles fastest
//     so the blocks that share an A row-panel share an L2.
#include <cstring>
#include "common.h"
#include "igemm.h"

namespace dpe {

constexpr int BK = 32;
constexpr int NT = 256;

// ---------------------------------------------------------------- LDS images
// K-contiguous image: row r holds 32 bf16 (64 B) as 4 chunks of 16 B.
DPE_DEVICE int kimg_off(int row, int chunk) {
  const int g = (0x78 >> (((row >> 2) & 3) << 1)) & 3;  // g = {0,2,3,1}
  return row * 64 + ((chunk ^ g) << 4);
}

// M/N-contiguous image: row k holds COLS bf16 as COLS/8 chunks of 16 B.
template <int COLS>
DPE_DEVICE int mnimg_off(int k, int chunk) {
  int h;
  if constexpr (COLS == 128 || COLS == 256) {
    // rows are whole multiples of the 256-B bank window, so the 128-column swizzle
    // (xor < 16 stays inside the row's first 16-chunk window) serves 256 columns too
    h = ((k & 3) | (((k >> 3) & 1) << 2)) << 1;
  } else {
    static_assert(COLS == 64, "mn image supports 64/128/256 columns");
    h = (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
  }
  return k * (COLS * 2) + ((chunk ^ h) << 4);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

DPE_DEVICE bf16x8 kfrag(const char* img, int r0) {
  const int lane = threadIdx.x & 63;
  const int row = r0 + (lane & 15);
  u32x4 v = *(const u32x4*)(img + kimg_off(row, lane >> 4));
  return __builtin_bit_cast(bf16x8, v);
}

template <int COLS>
DPE_DEVICE bf16x8 mnfrag(const char* img, int c0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k1 = 8 * g + q, k2 = k1 + 4;
  const int mc = (c0 >> 3) + (p >> 1);
  const int sub = (p & 1) * 8;
  const char* a1 = img + mnimg_off<COLS>(k1, mc) + sub;
  const char* a2 = img + mnimg_off<COLS>(k2, mc) + sub;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a2));
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8, r);
}

DPE_DEVICE u32x4 ld16(const uint16_t* p) { return *(const u32x4*)p; }
DPE_DEVICE u32x4 zero16() { u32x4 z; z[0] = z[1] = z[2] = z[3] = 0u; return z; }

// Out-of-range chunks (conv padding, M/N/K tails) load from this zero page: the
// address is selected (v_cndmask), the load is unconditional -- no branch per chunk.
__device__ __attribute__((aligned(64))) uint16_t igemm_zero_page[32];
DPE_DEVICE u32x4 ld16z(bool v, const uint16_t* p) { return *(const u32x4*)(v ? p : igemm_zero_page); }

// ------------------------------------------------------------------ loaders
// K-contiguous loaders: tile [ROWS][32]; chunk c -> row c>>2, kchunk c&3.
template <int ROWS, int KIND>
struct KLoader {
  static constexpr int NC = ROWS * 4 / NT;  // chunks per thread
  const uint16_t* base[NC];
  int row[NC];
  bool vrow[NC];
  // conv state per chunk
  int ihb[NC], iwb[NC];   // fwd: oh*sh-ph, ow*sw-pw ; dgrad: h+ph, w+pw
  int ci[NC], s[NC], r[NC];
  int kk[NC];             // absolute k of the chunk

  DPE_DEVICE void init(const IgemmArgs& p, const uint16_t* ptr, int64_t ld, int rows_total, int r0, int kb) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      row[i] = c >> 2;
      const int kc = c & 3;
      const int gr = r0 + row[i];
      vrow[i] = gr < rows_total;
      kk[i] = kb + kc * 8;
      if constexpr (KIND == A_DENSE_K || KIND == B_DENSE_K) {
        base[i] = ptr + (int64_t)(vrow[i] ? gr : 0) * ld + kk[i];
      } else {
        const ConvGeom& g = p.g;
        const int grr = vrow[i] ? gr : 0;
        if constexpr (KIND == A_CONV_FWD) {
          const int ow = grr % g.OW, t = grr / g.OW, oh = t % g.OH, n = t / g.OH;
          ihb[i] = oh * g.sh - g.ph;
          iwb[i] = ow * g.sw - g.pw;
          base[i] = ptr + (int64_t)n * g.H * g.W * g.C;
          const int kc0 = kk[i];
          ci[i] = kc0 % g.C;
          const int rs = kc0 / g.C;
          s[i] = rs % g.S;
          r[i] = rs / g.S;
        } else {  // A_CONV_DGRAD: rows over input pixels, k = (r, s, co)
          const int w = grr % g.W, t = grr / g.W, h = t % g.H, n = t / g.H;
          ihb[i] = h + g.ph;
          iwb[i] = w + g.pw;
          base[i] = ptr + (int64_t)n * g.OH * g.OW * g.K;
          const int kc0 = kk[i];
          ci[i] = kc0 % g.K;
          const int rs = kc0 / g.K;
          s[i] = rs % g.S;
          r[i] = rs / g.S;
        }
      }
    }
  }

  DPE_DEVICE void load(const IgemmArgs& p, int kend, u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      bool v = vrow[i] && kk[i] < kend;
      if constexpr (KIND == A_DENSE_K || KIND == B_DENSE_K) {
        regs[i] = ld16z(v, base[i]);
      } else if constexpr (KIND == A_CONV_FWD) {
        const ConvGeom& g = p.g;
        const int ih = ihb[i] + r[i] * g.dh, iw = iwb[i] + s[i] * g.dw;
        v = v && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        regs[i] = ld16z(v, base[i] + ((int64_t)ih * g.W + iw) * g.C + ci[i]);
      } else {  // A_CONV_DGRAD
        const ConvGeom& g = p.g;
        const int oh_ = ihb[i] - r[i] * g.dh, ow_ = iwb[i] - s[i] * g.dw;
        const int oh = oh_ / g.sh, ow = ow_ / g.sw;
        v = v && oh_ >= 0 && ow_ >= 0 && oh * g.sh == oh_ && ow * g.sw == ow_ && oh < g.OH && ow < g.OW;
        regs[i] = ld16z(v, base[i] + ((int64_t)oh * g.OW + ow) * g.K + ci[i]);
      }
    }
  }

  DPE_DEVICE void advance(const IgemmArgs& p) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      kk[i] += BK;
      if constexpr (KIND == A_DENSE_K || KIND == B_DENSE_K) {
        base[i] += BK;
      } else {
        const int C = (KIND == A_CONV_FWD) ? p.g.C : p.g.K;
        ci[i] += BK;
        while (ci[i] >= C) {
          ci[i] -= C;
          if (++s[i] == p.g.S) { s[i] = 0; ++r[i]; }
        }
      }
    }
  }

  DPE_DEVICE void store(char* img, const u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      *(u32x4*)(img + kimg_off(row[i], c & 3)) = regs[i];
    }
  }
};

// M/N-contiguous loaders: tile [32][COLS]; chunk c -> krow c/(COLS/8), col chunk c%(COLS/8).
template <int COLS, int KIND>
struct MNLoader {
  static constexpr int CPR = COLS / 8;
  static constexpr int NC = BK * CPR / NT;
  const uint16_t* base[NC];
  int krow[NC], cc[NC];
  bool vcol[NC];
  int kk[NC];
  // dgrad weights: k = (t,u,co) -> co, virtual taps (t,u) -> real (r,s)
  int co[NC], tt[NC], uu[NC];
  // wgrad im2col: k = pixel -> (img, oh, ow); column chunk -> (r, s, ci)
  int img[NC], oh[NC], ow[NC];
  int roff[NC], soff[NC];

  DPE_DEVICE void init(const IgemmArgs& p, const uint16_t* ptr, int64_t ld, int cols_total, int c0, int kb) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      krow[i] = c / CPR;
      cc[i] = c % CPR;
      const int gc = c0 + cc[i] * 8;
      vcol[i] = gc < cols_total;
      const int gcc = vcol[i] ? gc : 0;
      kk[i] = kb + krow[i];
      if constexpr (KIND == A_DENSE_M || KIND == B_DENSE_N) {
        base[i] = ptr + (int64_t)kk[i] * ld + gcc;
      } else if constexpr (KIND == B_CONV_DGRAD) {
        const ConvGeom& g = p.g;
        co[i] = kk[i] % g.K;
        const int rs = kk[i] / g.K;
        tt[i] = rs / g.S;
        uu[i] = rs % g.S;
        base[i] = ptr + gcc;  // + co*RR*SS*C + (r*SS + s)*C
      } else {  // B_CONV_WGRAD
        const ConvGeom& g = p.g;
        const int cin = gcc % g.C, t = gcc / g.C;
        const int ss = t % g.S, rr = t / g.S;
        roff[i] = rr * g.dh - g.ph;
        soff[i] = ss * g.dw - g.pw;
        base[i] = ptr + cin;
        const int px = kk[i];
        ow[i] = px % g.OW;
        const int tt = px / g.OW;
        oh[i] = tt % g.OH;
        img[i] = tt / g.OH;
      }
    }
  }

  DPE_DEVICE void load(const IgemmArgs& p, int kend, u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      bool v = vcol[i] && kk[i] < kend;
      if constexpr (KIND == A_DENSE_M || KIND == B_DENSE_N) {
        regs[i] = ld16z(v, base[i]);
      } else if constexpr (KIND == B_CONV_DGRAD) {
        const ConvGeom& g = p.g;
        const int r = g.pr0 + g.psh * tt[i], s_ = g.ps0 + g.psw * uu[i];
        regs[i] = ld16z(v, base[i] + (int64_t)co[i] * g.RR * g.SS * g.C + (int64_t)(r * g.SS + s_) * g.C);
      } else {
        const ConvGeom& g = p.g;
        const int ih = oh[i] * g.sh + roff[i], iw = ow[i] * g.sw + soff[i];
        v = v && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        regs[i] = ld16z(v, base[i] + (((int64_t)img[i] * g.H + ih) * g.W + iw) * g.C);
      }
    }
  }

  DPE_DEVICE void advance(const IgemmArgs& p, int64_t ld) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      kk[i] += BK;
      if constexpr (KIND == A_DENSE_M || KIND == B_DENSE_N) {
        base[i] += BK * ld;
      } else if constexpr (KIND == B_CONV_DGRAD) {
        co[i] += BK;
        while (co[i] >= p.g.K) {
          co[i] -= p.g.K;
          if (++uu[i] == p.g.S) { uu[i] = 0; ++tt[i]; }
        }
      } else {
        ow[i] += BK;
        while (ow[i] >= p.g.OW) {
          ow[i] -= p.g.OW;
          if (++oh[i] == p.g.OH) { oh[i] = 0; ++img[i]; }
        }
      }
    }
  }

  DPE_DEVICE void store(char* img_, const u32x4* regs) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) *(u32x4*)(img_ + mnimg_off<COLS>(krow[i], cc[i])) = regs[i];
  }
};

template <int KIND> struct IsK { static constexpr bool v = (KIND == A_DENSE_K || KIND == A_CONV_FWD || KIND == A_CONV_DGRAD); };
template <int KIND> struct IsBK { static constexpr bool v = (KIND == B_DENSE_K); };

DPE_DEVICE float act_fn(float x, int act) {
  if (act == ACT_RELU) return fmaxf(x, 0.f);
  if (act == ACT_GELU) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u = k0 * (x + k1 * x * x * x);
    return 0.5f * x * (1.f + tanhf(u));
  }
  return x;
}

// Shared bf16 epilogue (EPI_BF16 / EPI_BF16_BNB) of the implicit-GEMM kernels: stage the
// tile through LDS, then coalesced 16-B row stores with residual add and BatchNorm partials.
// acc[RM][RN] is one wave's (16 RM) x (16 RN) sub-tile at (wm, wn); NTH threads.  BatchNorm
// partials are always per 128-row (64 for BM = 64) sub-tile, so the partial layout does not
// depend on which kernel / tile ran: column (tm * NSUB + sub) of [2][N][stats_ld].
template <int BM, int BN, int RM, int RN, int NTH, int EPI>
DPE_DEVICE void epilogue_bf16(const IgemmArgs& p, float alpha, f32x4 (&acc)[RM][RN], char* smem, int m0, int n0, int tm,
                              int wm, int wn) {
  constexpr int CROW = BN * 2 + 16;
  constexpr int NW = NTH / 64;
  constexpr int SUBM = BM < 128 ? BM : 128, NSUB = BM / SUBM;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lm = lane & 15, ln4 = (lane >> 4) * 4;
  const int tilesSub = (p.M + SUBM - 1) / SUBM;
  constexpr bool BNB = (EPI == EPI_BF16_BNB);
  // Stage bf16 tile in LDS (row stride CROW), then coalesced 16-B stores.  Without bias and activation
  // (every conv epilogue) the staging is alpha * acc and the pack: the general path's per-element bias
  // test (a masked load, then a full vmcnt wait) and activation switch (the GELU branch is inlined per
  // element) were most of the epilogue's VALU / SALU instructions -- the short-K parity data grads of
  // strided convs, which store 4x the rows per MFMA of a stride-1 conv, ran epilogue-bound.
  if (!p.bias && p.act == ACT_NONE) {  // (uniform)
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int ml = wm + 16 * i + lm;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int nl = wn + 16 * j + ln4;
        u32x2 pk;
        pk[0] = pack_bf2(alpha * acc[i][j][0], alpha * acc[i][j][1]);
        pk[1] = pack_bf2(alpha * acc[i][j][2], alpha * acc[i][j][3]);
        *(u32x2*)(smem + ml * CROW + nl * 2) = pk;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int ml = wm + 16 * i + lm;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int nl = wn + 16 * j + ln4;
        const int n = n0 + nl;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float b = (p.bias && n + e < p.N) ? p.bias[n + e] : 0.f;
          v[e] = act_fn(alpha * acc[i][j][e] + b, p.act);
        }
        u32x2 pk;
        pk[0] = pack_bf2(v[0], v[1]);
        pk[1] = pack_bf2(v[2], v[3]);
        *(u32x2*)(smem + ml * CROW + nl * 2) = pk;
      }
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8, RPP = NTH / CPR;
  static_assert(SUBM % RPP == 0, "row passes must tile a stats sub-tile");
  const int c = tid % CPR, r0 = tid / CPR;
  const int n = n0 + c * 8;
  uint16_t* C = (uint16_t*)p.C;
  const bool vec = ((p.ldc & 7) == 0) && (n + 8 <= p.N);
  float s[8], ss[8];
  float bsc[8], bsh[8], bmu[8];  // BN forward coefficients of this thread's 8 columns (EPI_BF16_BNB)
  if constexpr (BNB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ch = min(n + e, p.N - 1);
      bsc[e] = p.st_coef[ch];
      bsh[e] = p.st_coef[p.N + ch];
      bmu[e] = p.st_coef[2 * p.N + ch];
    }
  }
  // Per-row finish: residual add, BN-backward partials / ReLU-mask (BNB) or BN-forward
  // partials, store.  Operands arrive pre-loaded (rv / xv / mb) so the fast path can
  // issue the loads of several rows before the first use.
  auto finish_row = [&](u32x4 v, const u32x4& rv, const u32x4& xv_raw, uint32_t mb, uint32_t rmb, uint16_t* dst,
                        bool vec_row) {
    if (p.residual) {
      float f[8], g[8];
      unpack8(v, f);
      unpack8(rv, g);
      if (p.res_mask) {  // residual = dy * relu'(y) from y's mask bits (dz never materialised)
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = ((rmb >> e) & 1u) ? g[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] += g[e];
      v = pack8(f);
    }
    if (p.col_stats) {
      float f[8];
      unpack8(v, f);
      if constexpr (BNB) {  // (sum dz, sum dz*(x - mean)), dz = f * relu'(...)
        float xv[8];
        unpack8(xv_raw, xv);
        if (p.st_mask) {  // relu'(y) from the saved post-residual output's mask bits; store dz itself
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            f[e] = ((mb >> e) & 1u) ? f[e] : 0.f;
            s[e] += f[e];
            ss[e] += f[e] * (xv[e] - bmu[e]);
          }
          v = pack8(f);
        } else {  // relu'(x*scale + shift), recomputed from the pre-BN input
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = fmaf(xv[e], bsc[e], bsh[e]) > 0.f ? f[e] : 0.f;
            s[e] += dz;
            ss[e] += dz * (xv[e] - bmu[e]);
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) { s[e] += f[e]; ss[e] += f[e] * f[e]; }
      }
    }
    if (vec_row) {
      *(u32x4*)dst = v;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (n + e < p.N) dst[e] = (uint16_t)((e & 1) ? (v[e >> 1] >> 16) : (v[e >> 1] & 0xffff));
      }
    }
  };
  constexpr int RPS = SUBM / RPP;               // rows per thread per stats sub-tile
  constexpr int G = RPS < 4 ? RPS : 4;          // rows whose operand loads are issued together
  const u32x4 z4 = zero16();
  // output row of tile row m: itself, or (phase data grads of strided convs) the real dX pixel of the
  // virtual row (n, hh, ww) -- remap 1: dgrad-form geometry (virtual output = H x W); 2: forward-form
  // (OH x OW).  The remapped rows take the batched path too: one row at a time, each waiting for its own
  // pre-BN / residual load, put the strided 3x3 data grads' epilogues at ~3x their streaming time
  // (4 phase launches of 52-157 us where the output bytes alone take ~17-50 us).
  auto orow_of = [&](int m) -> int64_t {
    if (!p.g.remap) return m;
    const int VW = p.g.remap == 2 ? p.g.OW : p.g.W, VH = p.g.remap == 2 ? p.g.OH : p.g.H;
    const int ww = m % VW, t = m / VW, hh = t % VH, nn = t / VH;
    return ((int64_t)nn * p.g.Hr + p.g.oa + p.g.psh * hh) * p.g.Wr + p.g.ob + p.g.psw * ww;
  };
  const bool fast = vec && m0 + BM <= p.M;
#pragma unroll
  for (int sub = 0; sub < NSUB; ++sub) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
    const int rb = sub * SUBM;
    if (fast) {
      // full tile: G rows' residual / pre-BN / mask loads in flight at once
#pragma unroll
      for (int u0 = 0; u0 < RPS; u0 += G) {
        u32x4 rv[G], xv[G];  // (the staged tile is read from LDS at the row's finish: fewer live registers)
        uint32_t mb[G], rmb[G];
        int64_t offs[G];
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const int rr = rb + r0 + (u0 + q) * RPP;
          const int64_t off = orow_of(m0 + rr) * p.ldc + n;
          offs[q] = off;
          rv[q] = p.residual ? (p.res_nt ? __builtin_nontemporal_load((const u32x4*)(p.residual + off))
                                         : ld16(p.residual + off))
                             : z4;
          xv[q] = (BNB && p.col_stats) ? ld16(p.st_x + off) : z4;
          mb[q] = (BNB && p.st_mask) ? (uint32_t)p.st_mask[off >> 3] : 0u;
          rmb[q] = p.res_mask ? (uint32_t)p.res_mask[off >> 3] : 0u;
        }
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const int rr = rb + r0 + (u0 + q) * RPP;
          finish_row(*(const u32x4*)(smem + rr * CROW + c * 16), rv[q], xv[q], mb[q], rmb[q], C + offs[q], true);
        }
      }
    } else {
      for (int rr = rb + r0; rr < rb + SUBM; rr += RPP) {
        const int m = m0 + rr;
        if (m >= p.M) break;
        const u32x4 v = *(const u32x4*)(smem + rr * CROW + c * 16);
        const int64_t off = orow_of(m) * p.ldc + n;
        u32x4 rv = z4, xv = z4;
        uint32_t mb = 0;
        if (vec) {
          if (p.residual) rv = ld16(p.residual + off);
          if (BNB && p.col_stats) xv = ld16(p.st_x + off);
        } else {
          float g[8], xf[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            g[e] = (p.residual && n + e < p.N) ? bf2f(p.residual[off + e]) : 0.f;
            xf[e] = (BNB && p.col_stats && n + e < p.N) ? bf2f(p.st_x[off + e]) : 0.f;
          }
          rv = pack8(g);
          xv = pack8(xf);
        }
        if (BNB && p.st_mask) mb = p.st_mask[off >> 3];
        const uint32_t rmb = p.res_mask ? (uint32_t)p.res_mask[off >> 3] : 0u;
        finish_row(v, rv, xv, mb, rmb, C + off, vec);
      }
    }
    if (p.col_stats) {
      // reduce over threads sharing column chunk c: lanes c + CPR*t within a wave, then NW waves via LDS
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = CPR; o < 64; o <<= 1) {
          s[e] += __shfl_xor(s[e], o, 64);
          ss[e] += __shfl_xor(ss[e], o, 64);
        }
      }
      float* red = (float*)(smem + BM * CROW);  // [2][NW][BN]
      if (sub > 0) __syncthreads();             // previous sub-tile's readers are done
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[wid * BN + c * 8 + e] = s[e];
          red[NW * BN + wid * BN + c * 8 + e] = ss[e];
        }
      }
      __syncthreads();
      // per-(M sub-tile) partials, layout [2][N][stats_ld]: no atomics, deterministic;
      // the BatchNorm finalize reduces the partials of each channel.
      const int col = tm * NSUB + sub;
      if (tid < BN && n0 + tid < p.N && col < tilesSub) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) { a += red[w * BN + tid]; b += red[NW * BN + w * BN + tid]; }
        const int sld = p.stats_ld ? p.stats_ld : tilesSub;
        p.col_stats[(int64_t)(n0 + tid) * sld + p.stats_off + col] = a;
        p.col_stats[(int64_t)(p.N + n0 + tid) * sld + p.stats_off + col] = b;
      }
    }
  }
}

// Split-K / accumulate epilogue (EPI_ATOMIC_F32) of the 2x2-wave kernels: stage the fp32 tile
// through LDS, half the rows at a time (the two wave-rows take turns), then add it with
// atomics shaped as whole contiguous row segments: every wave-instruction covers 64
// consecutive floats (256 B) of one row -- the full-rate atomic shape (MI355X_MICROARCH
// "Global float atomics"); a 16-rows x 4-dwords shape runs ~17x slower.
template <int BM, int BN, int LDS, int WGM = 2, int WGN = 2>
DPE_DEVICE void epilogue_atomic_f32(const IgemmArgs& p, f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16], char* smem, int m0,
                                    int n0, int wn, int split = 0) {
  constexpr int RM = BM / WGM / 16, RN = BN / WGN / 16, NW = WGM * WGN;
  constexpr int HR = BM / WGM;        // rows per pass (one wave-row at a time)
  constexpr int FROW = BN + 4;        // fp32 row stride (pad: conflict-free b128 writes)
  static_assert(HR * FROW * 4 <= LDS, "atomic staging must fit the kernel's LDS");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lm = lane & 15, ln4 = (lane >> 4) * 4;
  // p.slab: this split's partial tile is stored (plain, same row-segment shape) into its own slab
  float* const slab = p.slab ? p.slab + (int64_t)split * p.M * p.N : nullptr;
  float* C = (float*)p.C;
  float* st = (float*)smem;
#pragma unroll
  for (int half = 0; half < WGM; ++half) {
    if ((wid / WGN) == half) {
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int ml = 16 * i + lm;  // row within this pass
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const int nl = wn + 16 * j + ln4;
          *(f32x4*)(st + ml * FROW + nl) = acc[i][j] * p.alpha;
        }
      }
    }
    __syncthreads();
    constexpr int SEG = 64;                   // floats per wave-instruction
    constexpr int SEGS_PER_ROW = BN / SEG;    // 1, 2 or 4
    for (int s = wid; s < HR * SEGS_PER_ROW; s += NW) {
      const int r = s / SEGS_PER_ROW, c = (s % SEGS_PER_ROW) * SEG + lane;
      const int m = m0 + half * HR + r, n = n0 + c;
      if (m < p.M && n < p.N) {
        if (slab) slab[(int64_t)m * p.N + n] = st[r * FROW + c];
        else atomicAdd(C + (int64_t)m * p.ldc + n, st[r * FROW + c]);
      }
    }
    __syncthreads();
  }
}

// -------------------------------------------------------------------- kernel
#ifndef DPE_IGEMM_OCC4
#define DPE_IGEMM_OCC4 0
#endif
template <int BM, int BN, int AL, int BL, int EPI>
__global__ __launch_bounds__(NT, DPE_IGEMM_OCC4 ? 4 : 1) void igemm_kernel(IgemmArgs p) {
  constexpr bool AK = IsK<AL>::v;
  constexpr bool BKc = IsBK<BL>::v;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CROW = BN * 2 + 16;
  constexpr int LDS_MAIN = 2 * STAGE;
  constexpr int LDS_C = (EPI == EPI_BF16 || EPI == EPI_BF16_BNB) ? (BM * CROW + 2 * 4 * BN * 4)
                        : (EPI == EPI_ATOMIC_F32 ? (BM / 2) * (BN + 4) * 4 : 0);
  constexpr int LDS = LDS_MAIN > LDS_C ? LDS_MAIN : LDS_C;
  constexpr int RM = BM / 32, RN = BN / 32;
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tilesN = (p.N + BN - 1) / BN;
  const int tilesM = (p.M + BM - 1) / BM;
  const int ntile = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntile, split = bid / ntile;
  const int tm = tile / tilesN, tn = tile % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = split * p.k_split;
  const int ke = min(p.K, kb + p.k_split);
  const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);

  using ALdr = typename std::conditional<AK, KLoader<BM, AL>, MNLoader<BM, AL>>::type;
  using BLdr = typename std::conditional<BKc, KLoader<BN, BL>, MNLoader<BN, BL>>::type;
  ALdr al;
  BLdr bl;
  if constexpr (AK) al.init(p, p.A, p.lda, p.M, m0, kb); else al.init(p, p.A, p.lda, p.M, m0, kb);
  if constexpr (BKc) bl.init(p, p.B, p.ldb, p.N, n0, kb); else bl.init(p, p.B, p.ldb, p.N, n0, kb);

  u32x4 ra[ALdr::NC], rb[BLdr::NC];
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int cur = 0;
  if (kb < ke) {
    al.load(p, ke, ra);
    bl.load(p, ke, rb);
    al.store(smem, ra);
    bl.store(smem + A_BYTES, rb);
    if constexpr (AK) al.advance(p); else al.advance(p, p.lda);
    if constexpr (BKc) bl.advance(p); else bl.advance(p, p.ldb);
  }
  __syncthreads();

  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) {
      al.load(p, ke, ra);
      bl.load(p, ke, rb);
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      if constexpr (AK) af[i] = kfrag(As, wm + 16 * i);
      else af[i] = mnfrag<BM>(As, wm + 16 * i);
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      if constexpr (BKc) bfr[j] = kfrag(Bs, wn + 16 * j);
      else bfr[j] = mnfrag<BN>(Bs, wn + 16 * j);
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    if (more) {
      char* nxt = smem + (cur ^ 1) * STAGE;
      al.store(nxt, ra);
      bl.store(nxt + A_BYTES, rb);
      if constexpr (AK) al.advance(p); else al.advance(p, p.lda);
      if constexpr (BKc) bl.advance(p); else bl.advance(p, p.ldb);
    }
    __syncthreads();
    cur ^= 1;
  }

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][e]: m = m0 + wm + 16i + (lane&15), n = n0 + wn + 16j + (lane>>4)*4 + e
  if (p.alpha_ptr) p.alpha *= *p.alpha_ptr;
  const float alpha = p.alpha;
  const int lm = lane & 15, ln4 = (lane >> 4) * 4;
  if constexpr (EPI == EPI_ATOMIC_F32) {
    epilogue_atomic_f32<BM, BN, LDS>(p, acc, smem, m0, n0, wn);
    return;
  } else if constexpr (EPI == EPI_F32) {
    float* C = (float*)p.C;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int m = m0 + wm + 16 * i + lm;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int n = n0 + wn + 16 * j + ln4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float b = (p.bias && n + e < p.N) ? p.bias[n + e] : 0.f;
          v[e] = act_fn(alpha * acc[i][j][e] + b, p.act);
          if (p.residual_f32 && n + e < p.N) v[e] += p.residual_f32[(int64_t)m * p.ldc + n + e];
        }
        float* dst = C + (int64_t)m * p.ldc + n;
        if (n + 4 <= p.N && (p.ldc & 3) == 0) {
          *(f32x4*)dst = f32x4{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) if (n + e < p.N) dst[e] = v[e];
        }
      }
    }
    return;
  } else {
    epilogue_bf16<BM, BN, RM, RN, NT, EPI>(p, alpha, acc, smem, m0, n0, tm, wm, wn);
  }
}

// ------------------------------------------------- LDS-DMA conv / GEMM kernel
// Forward-form convolutions (and 1x1 / dense K-contiguous A) with operands
// streamed straight into LDS by buffer_load ... lds (no VGPR staging, no
// ds_write), a 3-stage ring (two K-steps of loads in flight behind the MFMAs)
// and one barrier per K-step.  Address work per K-step is scalar: with
// C % 32 == 0 a 32-wide K-step lies inside one filter tap, so the tap's byte
// offset goes in soffset, every lane keeps one 32-bit row offset (voffset) for
// the whole loop, and padding / tails come from a per-row tap-validity mask
// that swaps the offset for an out-of-range one (the buffer unit returns 0).
//
// B is [N][K] (BL == B_DENSE_K, K-image, ds_read_b128) or [K][N]
// (BL == B_DENSE_N, MN-image, ds_read_b64_tr_b16).  Shared epilogue.
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr uint32_t DMA_OOB = 0x80000000u;  // voffset past every buffer's num_records (< 2^31 bytes)
constexpr int DSTAGES = 3;

DPE_DEVICE __amdgpu_buffer_rsrc_t dma_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// LDS-DMA of one 16-B chunk per lane to wave_dst + 16 * lane.  Issued through inline asm: after a
// compiler-visible LDS-DMA, hipcc (ROCm 7.2) puts s_waitcnt vmcnt(0) in front of LDS reads it cannot
// prove disjoint from the DMA's destination (ds_read_b64_tr_b16 fragments, the A-transform's
// coefficient table), which drained the ring every K-step in the data-grad (B_DENSE_N) and the
// A-transform kernels.  The kernels' own counted wait_vm<N> calls order the DMA against the LDS
// reads; a VMEM op the compiler does not see can only make its own vmcnt waits stricter.  M0 is
// used by nothing else in these kernels.  (-DDPE_DMA_BUILTIN: the builtin, for A/B.)
DPE_DEVICE void dma16(__amdgpu_buffer_rsrc_t r, char* wave_dst, uint32_t voff, uint32_t soff) {
#ifdef DPE_DMA_BUILTIN
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)wave_dst, 16, voff, soff, 0, 0);
#else
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void_t*)wave_dst);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               ::"s"(m0), "v"(voff), "s"(r), "s"(soff) : "memory");
#endif
}

template <int N>
DPE_DEVICE void wait_vm() {
  // s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14; expcnt / lgkmcnt left at "no wait")
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
  asm volatile("" ::: "memory");
}

// WGM x WGN waves, each owning a (BM/WGM) x (BN/WGN) sub-tile; 128x128 (2x2 waves),
// 256x128 (4x2) and 256x256 (2x4).  Bigger tiles cut the L2->LDS bytes per FLOP, which
// bounds the 128-tile kernel (16 KiB per 256 MFMA-cycles per block).
#ifndef DPE_DMA_OCC4
#define DPE_DMA_OCC4 1  // hold the 4-wave tiles to 128 VGPRs: 4 blocks per CU even with the BN epilogue
                        // (a few epilogue spills; measured 44.2 -> 43.9 ms/step)
#endif
//
// AX != AX_NONE (dense A only, 2-stage ring): the A operand is the output of a BatchNorm pass that
// is never launched on its own (AXform, igemm.h) -- a second A tensor (a2) streams into the stage
// beside A, the per-K-channel coefficients are staged in LDS once, and the transformed fragments
// feed the MFMAs.  The waves of the first N tile whose columns start at 0 (exactly one wave per A row)
// also store the transformed A (and its ReLU-mask bits): the standalone pass that wrote it before
// read the same two tensors, so the consumer's own read of it is what disappears.
// The body is a device function of the block's (XCD-remapped) tile index `bid`: igemm_dma_kernel runs one
// problem, igemm_dma_group_kernel several of one shape class in one grid (the per-parity data grads of a
// strided conv).
template <int BM, int BN, int WGM, int WGN, int BL, int EPI, int NS = DSTAGES, int AX = AX_NONE>
DPE_DEVICE void igemm_dma_body(const IgemmArgs& p, int a_dense, const int bid) {
  constexpr int NTH = 64 * WGM * WGN, NW = WGM * WGN;
  constexpr bool BKc = (BL == B_DENSE_K);
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr bool CAT = AX == AX_CAT;
  constexpr int A2_BYTES = (AX && !CAT) ? A_BYTES : 0;
  static_assert(AX == AX_NONE || NS == 2, "A transform: 2-stage ring");
  constexpr int STAGE = A_BYTES + A2_BYTES + B_BYTES;
  constexpr int CROW = BN * 2 + 16;
  constexpr int LDS_MAIN = (NS == 4 ? 3 : NS) * STAGE;
  constexpr int LDS_C = BM * CROW + 2 * NW * BN * 4;
  constexpr int LDS = LDS_MAIN > LDS_C ? LDS_MAIN : LDS_C;
  constexpr int RM = BM / WGM / 16, RN = BN / WGN / 16;
  constexpr int PA = BM / (16 * NW), PB = BN / (16 * NW);  // 1-KiB DMA pieces per wave per stage
  static_assert(PA >= 1 && PB >= 1 && PA * 16 * NW == BM && PB * 16 * NW == BN, "DMA piece split");
  static_assert(BKc || BN <= 128, "MN image supports 64/128 columns");
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (p.N + BN - 1) / BN;
  const int tm = bid / tilesN, tn = bid % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = (wid / WGN) * (BM / WGM), wn = (wid % WGN) * (BN / WGN);
  const ConvGeom& g = p.g;
  const int C = a_dense ? p.K : g.C;  // channels per tap (the whole K for dense A)

  // ---- A rows: per-piece row offset + tap-validity mask (bit t = tap t in range)
  const bool c16 = !a_dense && g.C == 16;
  uint32_t aoff[PA], amask[PA], adsel[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = (wid * PA + i) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3);  // kimg swizzle (inverse = itself)
    const int m = m0 + row;
    uint32_t mask = 0u, off = 0u;
    if (m < p.M) {
      if (a_dense) {
        off = (uint32_t)m * (uint32_t)p.lda * 2u;
        mask = 1u;
      } else {
        const int ow = m % g.OW, t = m / g.OW, oh = t % g.OH, n = t / g.OH;
        const int ih0 = oh * g.sh - g.ph, iw0 = ow * g.sw - g.pw;
        off = (uint32_t)((((int64_t)n * g.H + oh * g.sh) * g.W + ow * g.sw) * g.C) * 2u;
        for (int r = 0; r < g.R; ++r) {
          const bool vr = (unsigned)(ih0 + r * g.dh) < (unsigned)g.H;
          for (int s = 0; s < g.S; ++s) {
            const bool vs = (unsigned)(iw0 + s * g.dw) < (unsigned)g.W;
            if (vr && vs) mask |= 1u << (r * g.S + s);
          }
        }
      }
    }
    // C = 16 (the s2d stem): a 32-wide K-step spans two taps; chunks 0-1 read tap t,
    // chunks 2-3 tap t+1 (adsel), each at channel offset (lc & 1) * 8
    aoff[i] = off + (c16 ? (lc & 1) : lc) * 16;
    amask[i] = mask;
    adsel[i] = c16 ? (lc >> 1) : 0;
  }
  // A's buffer starts (ph*W + pw)*C elements before x so that every in-range tap offset is >= 0
  const int64_t apre = a_dense ? 0 : ((int64_t)g.ph * g.W + g.pw) * g.C;
  const int64_t abytes = a_dense ? (int64_t)p.M * p.lda * 2 : ((int64_t)g.N * g.H * g.W * g.C + apre) * 2;
  const __amdgpu_buffer_rsrc_t ar = dma_rsrc(p.A - apre, (uint32_t)abytes);
  const __amdgpu_buffer_rsrc_t ar2 =
      CAT ? dma_rsrc(p.a2, (uint32_t)((int64_t)p.M * p.lda2 * 2)) : dma_rsrc(AX ? p.a2 : p.A, (uint32_t)abytes);
  // AX_CAT: the second segment's per-piece row offsets (dense rows, lda2)
  uint32_t aoff2[CAT ? PA : 1];
  if constexpr (CAT) {
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int row = (wid * PA + i) * 16 + (lane >> 2);
      const int lc = (lane & 3) ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3);
      const int m = m0 + row;
      aoff2[i] = m < p.M ? (uint32_t)m * (uint32_t)p.lda2 * 2u + lc * 16 : DMA_OOB;
    }
  }

  // ---- B: per-piece offsets, fixed for the loop (validity never changes along K)
  uint32_t boff[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int pc = wid * PB + i;
    if constexpr (BKc) {
      const int row = pc * 16 + (lane >> 2);
      const int lc = (lane & 3) ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3);
      const int n = n0 + row;
      boff[i] = n < p.N ? (uint32_t)(n * p.ldb + lc * 8) * 2u : DMA_OOB;
    } else {
      constexpr int CPR = BN / 8, KR = 64 / CPR;  // chunks per k-row, k-rows per piece
      const int krow = pc * KR + lane / CPR, ph_ = lane % CPR;
      int h;
      if constexpr (BN == 128) h = ((krow & 3) | (((krow >> 3) & 1) << 2)) << 1;
      else h = (((krow >> 1) & 1) | (((krow >> 3) & 1) << 1)) << 1;
      const int n = n0 + (ph_ ^ h) * 8;
      boff[i] = n < p.N ? (uint32_t)(krow * p.ldb + n) * 2u : DMA_OOB;
    }
  }
  const int64_t bbytes = BKc ? (int64_t)p.N * p.ldb * 2 : (int64_t)p.K * p.ldb * 2;
  const __amdgpu_buffer_rsrc_t br = dma_rsrc(p.B, (uint32_t)bbytes);
  const uint32_t bstep = BKc ? 64u : (uint32_t)p.ldb * 64u;  // bytes per K-step

  // ---- scalar K-walk state of the NEXT stage to issue
  int tap = 0, ci = 0, ts = 0;          // tap index, channel offset in tap, tap column s
  uint32_t tapoff = 0, kbo = 0;         // tap byte offset into A, K-step byte offset into B
  const uint32_t s_step = (uint32_t)g.dw * g.C * 2u, r_step = (uint32_t)g.dh * g.W * g.C * 2u;
  const int nt = p.K / BK;

  auto next_tap = [&]() {
    ++tap;
    if (++ts == (a_dense ? 1 : g.S)) {
      ts = 0;
      tapoff += r_step - (uint32_t)(g.S - 1) * s_step;
    } else {
      tapoff += s_step;
    }
  };
  auto issue = [&](int buf) {
    char* st = smem + buf * STAGE;
    if (c16) {  // taps (tap, tap + 1): per-lane tap select, offsets in voffset
      const uint32_t off1 = (ts + 1 == g.S) ? tapoff + r_step - (uint32_t)(g.S - 1) * s_step : tapoff + s_step;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int tl = tap + (int)adsel[i];
        const uint32_t v = ((amask[i] >> tl) & 1u) ? aoff[i] + (adsel[i] ? off1 : tapoff) : DMA_OOB;
        dma16(ar, st + (wid * PA + i) * 1024, v, 0u);
      }
    } else {
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const uint32_t v = ((amask[i] >> tap) & 1u) ? aoff[i] : DMA_OOB;
        if constexpr (CAT) {
          if (ci < p.k1) dma16(ar, st + (wid * PA + i) * 1024, v, ci * 2);
          else dma16(ar2, st + (wid * PA + i) * 1024, aoff2[i], (ci - p.k1) * 2);
        } else {
          dma16(ar, st + (wid * PA + i) * 1024, v, tapoff + ci * 2);
          if constexpr (AX != AX_NONE) dma16(ar2, st + A_BYTES + (wid * PA + i) * 1024, v, tapoff + ci * 2);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) dma16(br, st + A_BYTES + A2_BYTES + (wid * PB + i) * 1024, boff[i], kbo);
    kbo += bstep;
    if (c16) {
      next_tap();
      next_tap();
    } else {
      ci += BK;
      if (ci >= C) {
        ci = 0;
        next_tap();
      }
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A transform: the per-K-channel coefficient tables sit in (dynamic) LDS for the whole launch,
  // [NXC][K] floats (K <= 2048: <= 32 KiB, and the big-K shapes are the small-M ones); the lane
  // reads the 8 channels 32 t + 8 g .. +7 of each table per K-step (broadcast reads)
  constexpr int NXC = (AX == AX_BN_RES || CAT) ? 2 : AX == AX_BN_BWD ? 3 : 4;
  const int KT = CAT ? p.K - p.k1 : p.K;  // coefficient table length
  extern __shared__ __attribute__((aligned(16))) float ax_coef[];
  const int xg = (lane >> 4) * 8;
  // the waves holding output columns [0, BN/WGN) of the first N tile store the transformed A
  const bool ax_store = AX != AX_NONE && !CAT && tn == 0 && wn == 0;
  const __amdgpu_buffer_rsrc_t aout_r = dma_rsrc(AX ? (const void*)p.a_out : p.A, (uint32_t)((int64_t)p.M * p.lda * 2));
  const __amdgpu_buffer_rsrc_t bits_r = dma_rsrc(AX ? (const void*)p.a_bits : p.A, (uint32_t)((int64_t)p.M * p.lda / 8));
  auto xform_cat = [&](int t, bf16x8 (&a)[RM]) {
    // second segment, BN + ReLU on load: relu(a2 * s[k - k1] + t[k - k1])
    const int k = t * BK + xg - p.k1;
    float c[2][8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const f32x4 lo = *(const f32x4*)(ax_coef + q * KT + k), hi = *(const f32x4*)(ax_coef + q * KT + k + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { c[q][e] = lo[e]; c[q][e + 4] = hi[e]; }
    }
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      float f[8];
      unpack8(__builtin_bit_cast(u32x4, a[i]), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], c[0][e], c[1][e]), 0.f);
      a[i] = __builtin_bit_cast(bf16x8, pack8(f));
    }
  };
  auto xform = [&](int t, bf16x8 (&a)[RM], const bf16x8 (&a2)[RM]) {
    if constexpr (AX != AX_NONE && !CAT) {
      const int k = t * BK + xg;
      float c[NXC][8];
#pragma unroll
      for (int q = 0; q < NXC; ++q) {
        const f32x4 lo = *(const f32x4*)(ax_coef + q * p.K + k), hi = *(const f32x4*)(ax_coef + q * p.K + k + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { c[q][e] = lo[e]; c[q][e + 4] = hi[e]; }
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        float f[8], g[8];
        unpack8(__builtin_bit_cast(u32x4, a[i]), f);
        unpack8(__builtin_bit_cast(u32x4, a2[i]), g);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if constexpr (AX == AX_BN_RES) {
            f[e] = fmaxf(fmaf(f[e], c[0][e], c[1][e]) + g[e], 0.f);
          } else if constexpr (AX == AX_BN_RES2) {  // the residual rounded to bf16 first, as bn_apply2
            f[e] = fmaxf(fmaf(f[e], c[0][e], c[1][e]) + bf2f(f2bf(fmaf(g[e], c[2 % NXC][e], c[3 % NXC][e]))), 0.f);
          } else {
            f[e] = fmaf(c[0][e], f[e], fmaf(c[1 % NXC][e], g[e], c[2 % NXC][e]));
          }
        }
        const u32x4 pk = pack8(f);
        a[i] = __builtin_bit_cast(bf16x8, pk);
        if (ax_store) {
          // buffer stores, issued unconditionally (rows past M get an out-of-range offset and are
          // dropped by the buffer unit), so every storing wave has exactly AX_ST stores per K-step
          // behind the next stage's DMA -- the counted wait at the next step leaves them in flight
          const int m = m0 + wm + 16 * i + (lane & 15);
          const uint32_t off = (uint32_t)m * (uint32_t)p.lda + (uint32_t)k;  // elements (< 2^30: checked on the host)
          const bool ok = m < p.M;
          __builtin_amdgcn_raw_buffer_store_b128(pk, aout_r, ok ? off * 2u : DMA_OOB, 0, 0);
          if constexpr (AX != AX_BN_BWD) {
            // the row's 4 mask bytes of this K-step (lanes li, li+16, li+32, li+48) as one dword
            const uint32_t b = relu_mask_byte(pk), li = lane & 15;
            const uint32_t w = b | ((uint32_t)__shfl(b, li + 16, 64) << 8) | ((uint32_t)__shfl(b, li + 32, 64) << 16) |
                               ((uint32_t)__shfl(b, li + 48, 64) << 24);
            __builtin_amdgcn_raw_buffer_store_b32(w, bits_r, (ok && lane < 16) ? off >> 3 : DMA_OOB, 0, 0);
          }
        }
      }
    }
  };
  // stores per K-step of a storing wave (the counted wait below)
  constexpr int AX_ST = (AX == AX_NONE || CAT) ? 0 : AX == AX_BN_BWD ? RM : 2 * RM;
  if constexpr (AX != AX_NONE) {
    // tables: AX_BN_RES [scale | shift] = a_coef rows 0-1; AX_BN_BWD [a | b | c]; AX_BN_RES2 + a_coef2 rows 0-1;
    // AX_CAT [scale | shift] of the second segment's K - k1 channels (rows 0-1 of its [4][K - k1] BN coef)
    if (!CAT || p.a_coef) {
      for (int i = tid; i < NXC * KT; i += NTH) {
        const int q = i / KT, kk = i - q * KT;
        ax_coef[i] = (AX == AX_BN_RES2 && q >= 2) ? p.a_coef2[(q - 2) * KT + kk] : p.a_coef[q * KT + kk];
      }
      __syncthreads();
    }
  }

  auto read_frags = [&](int buf, bf16x8 (&a)[RM], bf16x8 (&b)[RN]) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES + A2_BYTES;
#pragma unroll
    for (int i = 0; i < RM; ++i) a[i] = kfrag(As, wm + 16 * i);
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      if constexpr (BKc) b[j] = kfrag(Bs, wn + 16 * j);
      else b[j] = mnfrag<BN>(Bs, wn + 16 * j);
    }
  };
  auto mfmas = [&](const bf16x8 (&a)[RM], const bf16x8 (&b)[RN]) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
  };
  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  {
    // NS-stage ring: stages t+1 .. t+NS-2 stay in flight while stage t is consumed
    // (a fragment-prefetch 3-buffer variant measured slower -- occupancy-bound: docs/perf_notes.md)
    static_assert(NS == 2 || NS == 3, "2- or 3-stage ring");
    if (nt > 0) issue(0);
    if (NS == 3 && nt > 1) issue(1);
    for (int t = 0; t < nt; ++t) {
      if (NS == 3 && t + 1 < nt) wait_vm<PA + PB>();
      else if (AX != AX_NONE && ax_store && t > 0) wait_vm<AX_ST>();  // the previous step's by-product stores stay in flight
      else wait_vm<0>();
      barrier();
      if (t + NS - 1 < nt) issue((t + NS - 1) % NS);
      bf16x8 af[RM], bfr[RN];
      read_frags(t % NS, af, bfr);
      if constexpr (CAT) {
        if (p.a_coef && t * BK >= p.k1) xform_cat(t, af);
      } else if constexpr (AX != AX_NONE) {
        bf16x8 a2f[RM];
        const char* A2s = smem + (t % NS) * STAGE + A_BYTES;
#pragma unroll
        for (int i = 0; i < RM; ++i) a2f[i] = kfrag(A2s, wm + 16 * i);
        xform(t, af, a2f);
      }
      mfmas(af, bfr);
    }
  }
  __syncthreads();
  const float alpha = p.alpha_ptr ? p.alpha * *p.alpha_ptr : p.alpha;  // (a local: no scratch copy of p)
  epilogue_bf16<BM, BN, RM, RN, NTH, EPI>(p, alpha, acc, smem, m0, n0, tm, wm, wn);
}

#define DPE_DMA_BOUNDS(BM, BN, WGM, WGN, AX)                                                                   \
  __launch_bounds__(64 * WGM * WGN, ((BM == 256 && BN == 128) || (DPE_DMA_OCC4 && WGM * WGN == 4))              \
                                        ? ((AX == AX_CAT && BN == 128) ? 3 : 4) : 1)
// (AX_CAT 128x128: 3 blocks per CU -- at 128 VGPRs its two-segment loader spilled 27 registers)
template <int BM, int BN, int WGM, int WGN, int BL, int EPI, int NS = DSTAGES, int AX = AX_NONE>
__global__ DPE_DMA_BOUNDS(BM, BN, WGM, WGN, AX) void igemm_dma_kernel(IgemmArgs p, int a_dense) {
  igemm_dma_body<BM, BN, WGM, WGN, BL, EPI, NS, AX>(p, a_dense, xcd_remap(blockIdx.x, gridDim.x));
}

// Several problems with the same tile count in one grid, interleaved: remapped block r runs tile r / n of
// problem r % n, so an XCD's consecutive blocks hold the n problems of neighbouring tiles -- the four parity
// sub-GEMMs of a strided data grad read the same dy rows (once from HBM, the rest from that XCD's L2) and
// store the interleaved pixels of the same dx rows at about the same time; one launch instead of n.
template <int BM, int BN, int WGM, int WGN, int BL, int EPI, int NS = DSTAGES>
__global__ DPE_DMA_BOUNDS(BM, BN, WGM, WGN, AX_NONE) void igemm_dma_group_kernel(IgemmGroup gp, int a_dense) {
  const int r = xcd_remap(blockIdx.x, gridDim.x);
  const int n = gp.n;
  igemm_dma_body<BM, BN, WGM, WGN, BL, EPI, NS, AX_NONE>(gp.a[r % n], a_dense, r / n);
}

// ------------------------------------------- LDS-DMA weight-grad (split-K) kernel
// dW[m = co][n] += sum_k dy[k][m] * B[k][n], k = output pixel: both operands are
// M/N-contiguous ([32][COLS] images, ds_read_b64_tr_b16 fragments) streamed by
// buffer_load ... lds into the same 3-stage ring as igemm_dma_kernel.  B is x
// itself (1x1 stride-1, B_DENSE_N) or the im2col of x (B_CONV_WGRAD): every
// lane's 8-column chunk is one (tap, channel-run) for the whole loop, and the
// pixel row it reads advances 32 pixels per K-step through an incremental
// (oh, ow, byte offset) walk -- no divisions in the loop, padding via the
// out-of-range offset.  fp32 atomic epilogue (split-K).
template <int COLS>
DPE_DEVICE int mn_swz(int k) {
  if constexpr (COLS >= 128) return ((k & 3) | (((k >> 3) & 1) << 2)) << 1;
  else return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
}

// 4 or 8 waves.  Tiles with 64x128 wave tiles (128x256 / 256x128 / 256x256: half the L2 bytes
// per flop of 128x128) measured 1.2-1.8x SLOWER on every ResNet-50 weight-grad shape
// (profiles/wgrad_bigtile_ab_r2.txt): at ~210 VGPRs they run 2 waves per SIMD where 128x128
// runs 4, and the one-barrier-per-32-K ring does not hide the DMA latency at that occupancy.
// Not instantiated; the waves-per-EU bound below is what such a tile needs.
template <int BM, int BN, int BL, int WGM = 2, int WGN = 2, int NS = DSTAGES>
// (the 4-wave tiles need <= 128 VGPRs for 4 waves per SIMD: a build of the 128x128 3x3 tile at 133 ran 1.3x
// slower; check scripts/isa_stats.py after edits -- a launch bound forcing it spilled the 1x1 tile instead)
__global__ __launch_bounds__(64 * WGM * WGN, (BN / WGN > 64) ? 2 : 1) void igemm_wgrad_dma_kernel(IgemmArgs p) {
  constexpr int NW = WGM * WGN;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr bool CONV = (BL == B_CONV_WGRAD);
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int LDS_MAIN = NS * STAGE, LDS_ST = (BM / WGM) * (BN + 4) * 4;
  constexpr int LDS = LDS_MAIN > LDS_ST ? LDS_MAIN : LDS_ST;
  constexpr int RM = BM / WGM / 16, RN = BN / WGN / 16;
  constexpr int PA = BM / (16 * NW), PB = BN / (16 * NW);  // 1-KiB pieces per wave per stage
  static_assert(PA >= 1 && PB >= 1, "every wave issues A and B pieces");
  constexpr int ACPR = BM / 8, AKR = 64 / ACPR, BCPR = BN / 8, BKR = 64 / BCPR;
  __shared__ __attribute__((aligned(16))) char smem[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (p.N + BN - 1) / BN, tilesM = (p.M + BM - 1) / BM;
  const int ntile = tilesM * tilesN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntile, split = bid / ntile;
  const int m0 = (tile / tilesN) * BM, n0 = (tile % tilesN) * BN;
  const int kb = split * p.k_split;
  const int ke = min(p.K, kb + p.k_split);
  const int nt = (ke - kb) / BK;
  const int wm = (wid / WGN) * (BM / WGM), wn = (wid % WGN) * (BN / WGN);
  const ConvGeom& g = p.g;

  // ---- A = dy [K][lda]: fixed per-lane offsets, scalar K-step offset
  uint32_t aoff[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int krow = (wid * PA + i) * AKR + lane / ACPR;
    const int m = m0 + ((lane % ACPR) ^ mn_swz<BM>(krow)) * 8;
    aoff[i] = m < p.M ? (uint32_t)(((int64_t)(kb + krow) * p.lda + m) * 2) : DMA_OOB;
  }
  const __amdgpu_buffer_rsrc_t ar = dma_rsrc(p.A, (uint32_t)((int64_t)p.K * p.lda * 2));
  const uint32_t astep = (uint32_t)p.lda * 64u;

  // ---- B
  uint32_t boff[PB];                      // dense: fixed offsets; conv: tap byte offset of the chunk
  int oh[PB], ow[PB], tr[PB], ts[PB];     // conv: pixel walk + tap displacement
  uint32_t roff[PB];                      // conv: byte offset of pixel (img, oh*sh, ow*sw)
  int64_t bpre = 0, bbytes;
  const uint32_t bstep = (uint32_t)p.ldb * 64u;
  if constexpr (CONV) {
    bpre = ((int64_t)g.ph * g.W + g.pw) * g.C;
    bbytes = ((int64_t)g.N * g.H * g.W * g.C + bpre) * 2;
  } else {
    bbytes = (int64_t)p.K * p.ldb * 2;
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int krow = (wid * PB + i) * BKR + lane / BCPR;
    const int gc = n0 + ((lane % BCPR) ^ mn_swz<BN>(krow)) * 8;
    if constexpr (CONV) {
      const bool vc = gc < p.N;
      const int gcc = vc ? gc : 0;
      const int ci = gcc % g.C, t = gcc / g.C;
      const int ss = t % g.S, rr = t / g.S;
      tr[i] = vc ? rr * g.dh - g.ph : -(1 << 28);  // invalid column: never in range
      ts[i] = ss * g.dw - g.pw;
      boff[i] = (uint32_t)((((int64_t)rr * g.dh * g.W + ss * g.dw) * g.C + ci) * 2);
      const int px = kb + krow;
      ow[i] = px % g.OW;
      const int q = px / g.OW;
      oh[i] = q % g.OH;
      const int img = q / g.OH;
      roff[i] = (uint32_t)((((int64_t)img * g.H + oh[i] * g.sh) * g.W + ow[i] * g.sw) * g.C * 2);
    } else {
      boff[i] = gc < p.N ? (uint32_t)(((int64_t)(kb + krow) * p.ldb + gc) * 2) : DMA_OOB;
    }
  }
  const __amdgpu_buffer_rsrc_t br = dma_rsrc(p.B - bpre, (uint32_t)bbytes);
  // per-step pixel advance of 32 = wa rows + wb columns (host guarantees wa + 1 <= OH)
  const int wa = CONV ? BK / g.OW : 0, wb = CONV ? BK % g.OW : 0;
  const uint32_t rs_ow = (uint32_t)g.sw * g.C * 2u, rs_oh = (uint32_t)g.sh * g.W * g.C * 2u;
  const uint32_t rs_img = (uint32_t)g.H * g.W * g.C * 2u;
  const uint32_t d_step = (uint32_t)wa * rs_oh + (uint32_t)wb * rs_ow;
  const uint32_t d_ow = rs_oh - (uint32_t)g.OW * rs_ow, d_oh = rs_img - (uint32_t)g.OH * rs_oh;

  uint32_t kso = 0;  // A / dense-B K-step byte offset of the next stage to issue
  auto issue = [&](int buf) {
    char* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < PA; ++i) dma16(ar, st + (wid * PA + i) * 1024, aoff[i], kso * astep);
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      if constexpr (CONV) {
        const bool v = (unsigned)(oh[i] * g.sh + tr[i]) < (unsigned)g.H && (unsigned)(ow[i] * g.sw + ts[i]) < (unsigned)g.W;
        dma16(br, st + A_BYTES + (wid * PB + i) * 1024, v ? roff[i] + boff[i] : DMA_OOB, 0u);
        // advance this lane's pixel by BK
        ow[i] += wb; oh[i] += wa; roff[i] += d_step;
        if (ow[i] >= g.OW) { ow[i] -= g.OW; oh[i] += 1; roff[i] += d_ow; }
        if (oh[i] >= g.OH) { oh[i] -= g.OH; roff[i] += d_oh; }
      } else {
        dma16(br, st + A_BYTES + (wid * PB + i) * 1024, boff[i], kso * bstep);
      }
    }
    ++kso;
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // b_coef (dense B only): BN + ReLU of B's producer on the fragments; a B fragment holds one
  // column (channel wn + 16 j + lane % 16) over 8 pixels.  Loaded before the ring's first DMA.
  const bool bnin = !CONV && p.b_coef != nullptr;
  float bsc[RN], bsh[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int n = min(n0 + wn + 16 * j + (lane & 15), p.N - 1);
    bsc[j] = bnin ? p.b_coef[n] : 1.f;
    bsh[j] = bnin ? p.b_coef[p.N + n] : 0.f;
  }

  // NS-stage ring: stages t+1 .. t+NS-2 stay in flight while stage t is consumed
  static_assert(NS == 2 || NS == 3, "2- or 3-stage ring");
  if (nt > 0) issue(0);
  if (NS == 3 && nt > 1) issue(1);
  for (int t = 0; t < nt; ++t) {
    if (NS == 3 && t + 1 < nt) wait_vm<PA + PB>(); else wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < nt) issue((t + NS - 1) % NS);
    const char* As = smem + (t % NS) * STAGE;
    const char* Bs = As + A_BYTES;
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = mnfrag<BM>(As, wm + 16 * i);
#pragma unroll
    for (int j = 0; j < RN; ++j) bfr[j] = mnfrag<BN>(Bs, wn + 16 * j);
    if (bnin) {
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        float f[8];
        unpack8(__builtin_bit_cast(u32x4, bfr[j]), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], bsc[j], bsh[j]), 0.f);
        bfr[j] = __builtin_bit_cast(bf16x8, pack8(f));
      }
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  }
  __syncthreads();
  if (p.alpha_ptr) p.alpha *= *p.alpha_ptr;
  epilogue_atomic_f32<BM, BN, LDS, WGM, WGN>(p, acc, smem, m0, n0, wn, split);
}

#ifndef DPE_WG_NS
#define DPE_WG_NS 2  // ring stages of the 4-wave weight-grad DMA tiles (compile-time A/B arm)
#endif

template <int BM, int BN, int AL, int BL, int EPI>
static void launch_t(const IgemmArgs& a, int splits, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((igemm_kernel<BM, BN, AL, BL, EPI>), dim3(tiles * splits), dim3(NT), 0, st, a);
}

template <int AL, int BL, int EPI>
static int launch_tiles(const IgemmArgs& a, int bm, int bn, int splits, hipStream_t st) {
  if (bm == 128 && bn == 128) launch_t<128, 128, AL, BL, EPI>(a, splits, st);
  else if (bm == 128 && bn == 64) launch_t<128, 64, AL, BL, EPI>(a, splits, st);
  else if (bm == 64 && bn == 128) launch_t<64, 128, AL, BL, EPI>(a, splits, st);
  else if (bm == 64 && bn == 64) launch_t<64, 64, AL, BL, EPI>(a, splits, st);
  else return -2;
  return 0;
}

}  // namespace dpe

using namespace dpe;

// Supported (aload, bload, epi) combinations — one per GEMM role.
extern "C" int dpe_igemm_launch(const IgemmArgs* args, int bm, int bn, int aload, int bload, int epi, int splits,
                                hipStream_t st) {
  const IgemmArgs& a = *args;
  if (a.M <= 0 || a.N <= 0) return 0;
  if (a.slab) return -1;  // slab partials: LDS-DMA weight grad only
  if (splits < 1) splits = 1;
#define DPE_CASE(AL, BL, EP) \
  if (aload == AL && bload == BL && epi == EP) return launch_tiles<AL, BL, EP>(a, bm, bn, splits, st);
  // dense Linear / 1x1 conv
  DPE_CASE(A_DENSE_K, B_DENSE_K, EPI_BF16)
  DPE_CASE(A_DENSE_K, B_DENSE_K, EPI_F32)
  DPE_CASE(A_DENSE_K, B_DENSE_N, EPI_BF16)
  DPE_CASE(A_DENSE_K, B_DENSE_N, EPI_F32)
  DPE_CASE(A_DENSE_M, B_DENSE_N, EPI_ATOMIC_F32)
  DPE_CASE(A_DENSE_M, B_DENSE_N, EPI_F32)
  // conv
  DPE_CASE(A_CONV_FWD, B_DENSE_K, EPI_BF16)
  DPE_CASE(A_CONV_DGRAD, B_CONV_DGRAD, EPI_BF16)
  // data-grad feeding a BN+ReLU backward (partials from the epilogue)
  DPE_CASE(A_DENSE_K, B_DENSE_N, EPI_BF16_BNB)
  DPE_CASE(A_CONV_DGRAD, B_CONV_DGRAD, EPI_BF16_BNB)
  DPE_CASE(A_CONV_FWD, B_DENSE_K, EPI_BF16_BNB)
  DPE_CASE(A_DENSE_M, B_CONV_WGRAD, EPI_ATOMIC_F32)
#undef DPE_CASE
  return -1;
}

// LDS-DMA kernel for forward-form convolutions / dense K-contiguous A.  Returns -1
// when the problem is outside its envelope (the caller then uses dpe_igemm_launch).
extern "C" int dpe_igemm_dma_launch(const IgemmArgs* args, int bm, int bn, int aload, int bload, int epi,
                                    hipStream_t st) {
  const IgemmArgs& a = *args;
  if (a.M <= 0 || a.N <= 0) return 0;
  if (aload != A_DENSE_K && aload != A_CONV_FWD) return -1;
  if (bload != B_DENSE_K && bload != B_DENSE_N) return -1;
  if (epi != EPI_BF16 && epi != EPI_BF16_BNB) return -1;
  if (a.K <= 0 || a.K % 32 || a.k_split < a.K) return -1;
  const bool dense = aload == A_DENSE_K;
  const ConvGeom& g = a.g;
  if (!dense && ((g.C % 32 && !(g.C == 16 && (g.R * g.S) % 2 == 0)) || g.R * g.S > 32 || g.R * g.S * g.C != a.K)) return -1;
  if (a.ldb % 8 || (bload == B_DENSE_N && a.N % 8) || (dense && a.lda % 8)) return -1;
  const int64_t lim = (1ll << 31) - 4096;
  const int64_t abytes = dense ? (int64_t)a.M * a.lda * 2
                               : ((int64_t)g.N * g.H * g.W * g.C + ((int64_t)g.ph * g.W + g.pw) * g.C) * 2;
  const int64_t bbytes = bload == B_DENSE_K ? (int64_t)a.N * a.ldb * 2 : (int64_t)a.K * a.ldb * 2;
  if (abytes >= lim || bbytes >= lim) return -1;
  const int tiles = ((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  const int dn = dense ? 1 : 0;
  if (a.a_mode == AX_CAT) {
    // concatenated-K data grad: A segments dense, K1 = k1 from A (lda), K - k1 from a2 (lda2)
    if (!dense || !a.a2 || a.k1 <= 0 || a.k1 % 32 || a.k1 >= a.K || a.lda < a.k1 || a.lda2 < a.K - a.k1 ||
        a.lda2 % 8 || (int64_t)a.M * a.lda2 * 2 >= lim || a.K - a.k1 > 2048)
      return -1;
#define DPE_DMA_CAT(BM_, BN_, WGM_, WGN_, BL_, EP_)                                                         \
  if (bm == BM_ && bn == BN_ && bload == BL_ && epi == EP_) {                                               \
    hipLaunchKernelGGL((igemm_dma_kernel<BM_, BN_, WGM_, WGN_, BL_, EP_, 2, AX_CAT>), dim3(tiles),          \
                       dim3(64 * WGM_ * WGN_), a.a_coef ? (size_t)2 * (a.K - a.k1) * 4 : 0, st, a, dn);     \
    return 0;                                                                                               \
  }
    DPE_DMA_CAT(128, 64, 2, 2, B_DENSE_N, EPI_BF16_BNB)
    DPE_DMA_CAT(128, 128, 2, 2, B_DENSE_N, EPI_BF16_BNB)
    DPE_DMA_CAT(128, 64, 2, 2, B_DENSE_N, EPI_BF16)
    DPE_DMA_CAT(128, 128, 2, 2, B_DENSE_N, EPI_BF16)
#undef DPE_DMA_CAT
    return -1;
  }
  if (a.a_mode != AX_NONE) {
    // A on-load transform: dense A with lda == K (the by-product is a whole [M][K] tensor)
    if (!dense || a.lda != a.K || !a.a2 || !a.a_coef || !a.a_out) return -1;
    if (a.a_mode == AX_BN_RES2 && !a.a_coef2) return -1;
    const int ncoef = a.a_mode == AX_BN_RES ? 2 : a.a_mode == AX_BN_BWD ? 3 : 4;
    if (a.K > 2048) return -1;  // coefficient tables <= 32 KiB of LDS
    if (a.a_mode != AX_BN_BWD && !a.a_bits) return -1;
    if ((int64_t)a.M * a.lda >= (1ll << 30)) return -1;  // 32-bit buffer offsets of the by-product
#define DPE_DMA_AX(BM_, BN_, WGM_, WGN_, BL_, EP_, AX_)                                                     \
  if (bm == BM_ && bn == BN_ && bload == BL_ && epi == EP_ && a.a_mode == AX_) {                            \
    hipLaunchKernelGGL((igemm_dma_kernel<BM_, BN_, WGM_, WGN_, BL_, EP_, 2, AX_>), dim3(tiles),             \
                       dim3(64 * WGM_ * WGN_), (size_t)ncoef * a.K * 4, st, a, dn);                         \
    return 0;                                                                                               \
  }
    // forward: the next block's conv1 over relu(BN3(h3) + identity) of the block before it
    DPE_DMA_AX(128, 64, 2, 2, B_DENSE_K, EPI_BF16, AX_BN_RES)
    DPE_DMA_AX(128, 128, 2, 2, B_DENSE_K, EPI_BF16, AX_BN_RES)
    DPE_DMA_AX(256, 64, 4, 1, B_DENSE_K, EPI_BF16, AX_BN_RES)
    DPE_DMA_AX(128, 64, 2, 2, B_DENSE_K, EPI_BF16, AX_BN_RES2)
    DPE_DMA_AX(128, 128, 2, 2, B_DENSE_K, EPI_BF16, AX_BN_RES2)
    DPE_DMA_AX(256, 64, 4, 1, B_DENSE_K, EPI_BF16, AX_BN_RES2)
    // backward: conv3's data grad over BN3's backward apply (dh3 = a dz3 + b h3 + c)
    DPE_DMA_AX(128, 64, 2, 2, B_DENSE_N, EPI_BF16_BNB, AX_BN_BWD)
    DPE_DMA_AX(128, 128, 2, 2, B_DENSE_N, EPI_BF16_BNB, AX_BN_BWD)
#undef DPE_DMA_AX
    return -1;
  }
// 4-wave tiles: a 2-stage ring keeps 4 blocks/CU; tiles up to DPE_DMA_NS3_MAX elements take the
// 3-stage ring (two K-steps in flight)
#ifndef DPE_DMA_NS3_MAX
#define DPE_DMA_NS3_MAX 0
#endif
#ifndef DPE_DMA_W64_NS2
#define DPE_DMA_W64_NS2 1  // 256x64: 2-stage ring (40 KiB, 4 blocks/CU) instead of 3 (60 KiB, 2)
#endif
#define DPE_DMA(BM_, BN_, WGM_, WGN_, BL_, EP_)                                                             \
  if (bm == BM_ && bn == BN_ && bload == BL_ && epi == EP_) {                                               \
    constexpr int NS_ = ((BM_ <= 128 && BN_ <= 128 && BM_ * BN_ > DPE_DMA_NS3_MAX) ||                        \
                         (BM_ == 256 && BN_ == 64 && DPE_DMA_W64_NS2)) ? 2 : 3;                                 \
    hipLaunchKernelGGL((igemm_dma_kernel<BM_, BN_, WGM_, WGN_, BL_, EP_, NS_>), dim3(tiles),                 \
                       dim3(64 * WGM_ * WGN_), 0, st, a, dn);                                               \
    return 0;                                                                                               \
  }
#define DPE_DMA_T(BL_, EP_) \
  DPE_DMA(128, 128, 2, 2, BL_, EP_) DPE_DMA(128, 64, 2, 2, BL_, EP_) DPE_DMA(64, 128, 2, 2, BL_, EP_) DPE_DMA(64, 64, 2, 2, BL_, EP_)
  DPE_DMA_T(B_DENSE_K, EPI_BF16)
  DPE_DMA_T(B_DENSE_K, EPI_BF16_BNB)
  DPE_DMA_T(B_DENSE_N, EPI_BF16)
  DPE_DMA_T(B_DENSE_N, EPI_BF16_BNB)
  // 8-wave big tiles (B K-contiguous)
  DPE_DMA(256, 128, 4, 2, B_DENSE_K, EPI_BF16)
  DPE_DMA(256, 128, 4, 2, B_DENSE_K, EPI_BF16_BNB)
  DPE_DMA(256, 256, 2, 4, B_DENSE_K, EPI_BF16)
  DPE_DMA(256, 256, 2, 4, B_DENSE_K, EPI_BF16_BNB)
  // 4-wave 256x64 (4x1 waves) for the N = 64 layers
  DPE_DMA(256, 64, 4, 1, B_DENSE_K, EPI_BF16)
  DPE_DMA(256, 64, 4, 1, B_DENSE_K, EPI_BF16_BNB)
#undef DPE_DMA_T
#undef DPE_DMA
  return -1;
}

extern "C" int dpe_igemm_dma_group_launch(const IgemmArgs* args, int n, int bm, int bn, int aload, int bload, int epi,
                                          hipStream_t st) {
  if (n < 1 || n > IGEMM_GROUP_MAX) return -1;
  if (aload != A_DENSE_K && aload != A_CONV_FWD) return -1;
  if (bload != B_DENSE_K || (epi != EPI_BF16 && epi != EPI_BF16_BNB)) return -1;
  const bool dense = aload == A_DENSE_K;
  const int64_t lim = (1ll << 31) - 4096;
  IgemmGroup gp;
  memset(&gp, 0, sizeof(gp));
  gp.n = n;
  for (int i = 0; i < n; ++i) {
    const IgemmArgs& a = args[i];
    // the single-problem launcher's envelope (dpe_igemm_dma_launch), no A transform, one tile count
    if (a.M <= 0 || a.N <= 0 || a.M != args[0].M || a.N != args[0].N || a.a_mode != AX_NONE) return -1;
    if (a.K <= 0 || a.K % 32 || a.k_split < a.K || a.ldb % 8 || (dense && a.lda % 8)) return -1;
    const ConvGeom& g = a.g;
    if (!dense && (g.C % 32 || g.R * g.S > 32 || g.R * g.S * g.C != a.K)) return -1;
    const int64_t abytes = dense ? (int64_t)a.M * a.lda * 2
                                 : ((int64_t)g.N * g.H * g.W * g.C + ((int64_t)g.ph * g.W + g.pw) * g.C) * 2;
    if (abytes >= lim || (int64_t)a.N * a.ldb * 2 >= lim) return -1;
    gp.a[i] = a;
  }
  const int tiles = ((args[0].M + bm - 1) / bm) * ((args[0].N + bn - 1) / bn);
  const int dn = dense ? 1 : 0;
#define DPE_DMA_G(BM_, BN_, WGM_, WGN_, NS_, EP_)                                                            \
  if (bm == BM_ && bn == BN_ && epi == EP_) {                                                                 \
    hipLaunchKernelGGL((igemm_dma_group_kernel<BM_, BN_, WGM_, WGN_, B_DENSE_K, EP_, NS_>), dim3(tiles * n),   \
                       dim3(64 * WGM_ * WGN_), 0, st, gp, dn);                                                \
    return 0;                                                                                                 \
  }
  DPE_DMA_G(128, 128, 2, 2, 2, EPI_BF16_BNB)
  DPE_DMA_G(128, 128, 2, 2, 2, EPI_BF16)
  DPE_DMA_G(256, 128, 4, 2, 3, EPI_BF16_BNB)
  DPE_DMA_G(256, 128, 4, 2, 3, EPI_BF16)
#undef DPE_DMA_G
  return -1;
}

// LDS-DMA weight-grad kernel (A = dy M-contiguous; B = x or im2col(x) N-contiguous;
// EPI_ATOMIC_F32, split-K).  -1: outside its envelope (caller uses dpe_igemm_launch).
extern "C" int dpe_igemm_wgrad_dma_launch(const IgemmArgs* args, int bm, int bn, int bload, int splits,
                                          hipStream_t st) {
  const IgemmArgs& a = *args;
  if (a.M <= 0 || a.N <= 0) return 0;
  if (bload != B_DENSE_N && bload != B_CONV_WGRAD) return -1;
  if (a.K <= 0 || a.K % 32 || a.k_split % 32 || a.M % 8 || a.N % 8 || a.lda % 8 || a.ldb % 8) return -1;
  const int64_t lim = (1ll << 31) - 4096;
  if ((int64_t)a.K * a.lda * 2 >= lim) return -1;
  const ConvGeom& g = a.g;
  if (bload == B_CONV_WGRAD) {
    if (g.C % 8 || (int64_t)g.N * g.OH * g.OW != a.K || g.R * g.S * g.C != a.N) return -1;
    if (32 / g.OW + 1 > g.OH) return -1;  // pixel walk: at most one image wrap per K-step
    if (((int64_t)g.N * g.H * g.W * g.C + ((int64_t)g.ph * g.W + g.pw) * g.C) * 2 >= lim) return -1;
  } else if ((int64_t)a.K * a.ldb * 2 >= lim) {
    return -1;
  }
  if (splits < 1) splits = 1;
  const int tiles = ((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
#define DPE_WG(BM_, BN_, BL_)                                                                                \
  if (bm == BM_ && bn == BN_ && bload == BL_) {                                                               \
    hipLaunchKernelGGL((igemm_wgrad_dma_kernel<BM_, BN_, BL_, 2, 2, DPE_WG_NS>), dim3(tiles * splits), dim3(NT), 0, st, a); \
    return 0;                                                                                                 \
  }
#define DPE_WG_T(BL_) DPE_WG(128, 128, BL_) DPE_WG(128, 64, BL_) DPE_WG(64, 128, BL_) DPE_WG(64, 64, BL_)
  DPE_WG_T(B_DENSE_N)
  DPE_WG_T(B_CONV_WGRAD)
  // Cout = 64 layers: one 64-row wave band, 4 waves across 256 columns
  if (bm == 64 && bn == 256 && bload == B_CONV_WGRAD) {
    hipLaunchKernelGGL((igemm_wgrad_dma_kernel<64, 256, B_CONV_WGRAD, 1, 4>), dim3(tiles * splits), dim3(NT), 0, st, a);
    return 0;
  }
#undef DPE_WG_T
#undef DPE_WG
  return -1;
}
