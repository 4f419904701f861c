// Narrow dense linears of the refine (K <= 128: the qkv / proj / pooling projections of the C <= 128 stages):
//
//   Y[m, n] = act(sum_k A[m, k] W[n, k] + bias[n]) + R[m, n]        (optionally publishing max |Y|)
//
// At K <= 128 a gemm_kernel tile has 2-4 K-slabs, so its fixed per-tile costs (prologue, LDS staging of both
// operands, epilogue at one tile per wave group) dominate and these launches ran at 25-100 TF/s, 2.5-3 TB/s
// of their HBM bytes (profiles/r03_gemm_calls.txt).  This kernel is built around the fact that W is small:
//   * a workgroup stages its 128-column block of the pre-split W (sfx_weight_split: fp16 h / l terms, per-row
//     scale) into LDS once -- 2 x 128 x K fp16 planes, rows swizzled for conflict-free ds_read_b128 -- and
//     then streams row tiles through it for the rest of the launch (persistent, grid-stride over 32-row tiles);
//   * each wave owns whole 32-row tiles and needs no workgroup barrier after the staging: the tile's A rows
//     are loaded straight into registers as MFMA B fragments (lane (r, h) holds row r's k = 16 t + 8 h .. + 7,
//     the fused MLP's layout, csrc/mlp.hip), the next tile's rows are in flight while the current one computes;
//   * per row one power-of-two scale from the exact row maximum (the whole row is in the lane pair), W rows
//     their own (from the split): D^T = W . A^T on v_mfma_f32_32x32x16_f16 as h*h + h*l + l*h with fp32
//     accumulation -- the GEMM family's fp32-accurate fp16x2 scheme;
//   * epilogue from the accumulator registers: a lane holds 4 x 4 consecutive output columns of one row,
//     so bias / GELU / residual / max |Y| are applied in registers and Y leaves by 16-byte stores.
// HBM traffic is the algorithmic A read (once per 128-column block) + R read + Y write.
#include <cstdlib>

#include "gemm_common.h"

namespace {

using namespace sfxg;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int NRW = 4;     // waves per workgroup
constexpr int NCOL = 128;  // output columns per workgroup (4 x 32)

// fp16 plane of the staged W block: [128 rows][KP] with KP = K rounded up to a power of two; the 16-byte chunk c
// (k = 8 c .. 8 c + 7) of row n sits at chunk c ^ ((n / (128 / KP)) & (KP / 8 - 1)), so the 16 rows one
// ds_read_b128 lane group reads cover all 64 banks once
template <int KP>
__device__ __forceinline__ int wchunk(int n, int c) {
  return n * (2 * KP) + ((c ^ ((n / (128 / KP)) & (KP / 8 - 1))) << 4);
}

template <int K>
__global__ void __launch_bounds__(NRW * 64, 2)
    gemm_narrow_kernel(int M, int N, const float* __restrict__ A, long long lda, const float* __restrict__ Wsp,
                       const float* __restrict__ winv, const float* __restrict__ bias, int act, int act_ncols,
                       const float* __restrict__ R, long long ldr, float* __restrict__ Y, long long ldy,
                       unsigned long long* __restrict__ y_amax, unsigned y_tag, int ncolblk, int nrowgrp) {
  constexpr int KP = K <= 64 ? 64 : 128;
  constexpr int KT = K / 16;               // k-steps
  constexpr int PLANE = NCOL * KP * 2;     // bytes per term plane
  __shared__ __attribute__((aligned(16))) char s_w[2 * PLANE];
  __shared__ float s_bias[NCOL], s_winv[NCOL], s_wave[NRW];

  // XCD-aware numbering: the column blocks of one row group are consecutive logical ids on one XCD, so the
  // A rows they all read come from that XCD's L2
  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8u) * (nb / 8) + (int)(blockIdx.x / 8u);
  const int cblk = L % ncolblk, rgrp = L / ncolblk;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int n0 = cblk * NCOL;
  const int ncb = min(4, (N - n0 + 31) / 32);  // 32-column blocks of this workgroup (wave-uniform)

  const __amdgpu_buffer_rsrc_t rA = rsrc_ext(A, (unsigned)M * (unsigned)lda * 4u);
  const __amdgpu_buffer_rsrc_t rY = rsrc_ext(Y, (unsigned)M * (unsigned)ldy * 4u);
  const __amdgpu_buffer_rsrc_t rR = rsrc_ext(R ? R : Y, R ? (unsigned)M * (unsigned)ldr * 4u : 0u);
  const int ntiles = (M + 31) / 32;
  const int tstride = nrowgrp * NRW;
  int tile = rgrp * NRW + wid;

  auto load_rows = [&](int t, float4 (&v)[2 * KT]) {
    const int m = t * 32 + r32;
    const unsigned base = (t < ntiles && m < M) ? (unsigned)m * (unsigned)lda : 0xffffffffu;
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      const unsigned c = (unsigned)(16 * s + 8 * h);
      v[2 * s] = bload4(rA, base != 0xffffffffu ? (base + c) * 4u : OOB);
      v[2 * s + 1] = bload4(rA, base != 0xffffffffu ? (base + c + 4u) * 4u : OOB);
    }
  };
  // the residual rows of tile t for every column block of this workgroup (loaded with the tile's A rows)
  auto load_res = [&](int t, float4 (&rv)[16]) {
    const int m = t * 32 + r32;
    const bool ok = R != nullptr && t < ntiles && m < M;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + cb * 32 + 8 * g + 4 * h;
        rv[4 * cb + g] = bload4(rR, (ok && cb < ncb && n < N) ? ((unsigned)m * (unsigned)ldr + (unsigned)n) * 4u : OOB);
      }
  };
  float4 vn[2 * KT];
  load_rows(tile, vn);  // the first tile's rows fly while W is staged

  // ---- stage the W block (pre-split rows n0 .. n0 + 127; rows past N zero) + its column constants ----
  {
    constexpr int GROUPS = NCOL * (K / 4);  // 4-element groups: 16 bytes of the split each (4 h then 4 l)
    const __amdgpu_buffer_rsrc_t rW = rsrc_ext(Wsp, (unsigned)N * (unsigned)K * 4u);
    for (int g = tid; g < GROUPS; g += NRW * 64) {
      const int n = g / (K / 4), k0 = 4 * (g - n * (K / 4));
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rW, (unsigned)((n0 + n) * K + k0) * 4u, 0, 0);
      const int off = wchunk<KP>(n, k0 >> 3) + ((k0 & 4) << 1);
      *reinterpret_cast<uint2*>(s_w + off) = make_uint2(v.x, v.y);
      *reinterpret_cast<uint2*>(s_w + PLANE + off) = make_uint2(v.z, v.w);
    }
    if (tid < NCOL) {
      const int n = n0 + tid;
      s_bias[tid] = (bias && n < N) ? bias[n] : 0.f;
      s_winv[tid] = n < N ? winv[n] : 0.f;
    }
  }
  __syncthreads();

  auto mfma3 = [](const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, floatx16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);  // smallest terms first
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  };

  float ymax = 0.f;
  for (; tile < ntiles; tile += tstride) {
    float4 v[2 * KT];
#pragma unroll
    for (int i = 0; i < 2 * KT; ++i) v[i] = vn[i];
    float4 rv[16];
    load_res(tile, rv);             // this tile's residual, needed only in the epilogues
    load_rows(tile + tstride, vn);  // the next tile's rows in flight during this one's MFMAs
    // row scale: the exact row maximum (this lane's half row + its partner's) in [2^13, 2^14)
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < 2 * KT; ++i)
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    int e = 0;
    if (mx > 0.f && mx <= 3.4028235e38f) e = row_exp(mx) + 1;
    const float sc = ldexpf(1.f, e), ainv = ldexpf(1.f, -e);
    f16x8 hb[KT][2];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      uint2 lo[2], hi[2];
      split2h(v[2 * s], sc, lo);
      split2h(v[2 * s + 1], sc, hi);
      hb[s][0] = __builtin_bit_cast(f16x8, make_uint4(lo[0].x, lo[0].y, hi[0].x, hi[0].y));
      hb[s][1] = __builtin_bit_cast(f16x8, make_uint4(lo[1].x, lo[1].y, hi[1].x, hi[1].y));
    }
    const int m = tile * 32 + r32;
    const bool mok = m < M;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      if (cb >= ncb) break;
      floatx16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
      const int wrow = cb * 32 + r32;
#pragma unroll
      for (int s = 0; s < KT; ++s) {
        const int off = wchunk<KP>(wrow, 2 * s + h);
        const f16x8 wh = *reinterpret_cast<const f16x8*>(s_w + off);
        const f16x8 wl = *reinterpret_cast<const f16x8*>(s_w + PLANE + off);
        acc = mfma3(wh, wl, hb[s][0], hb[s][1], acc);
      }
      // D^T layout: register i of lane half h = output column cb*32 + (i & 3) + 8 (i >> 2) + 4 h of row m
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = cb * 32 + 8 * g + 4 * h;  // column within the block
        const int n = n0 + c;
        float y[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float t = acc[4 * g + q] * (ainv * s_winv[c + q]) + s_bias[c + q];
          if (act == ACT_GELU && n + q < act_ncols) t = gelu_erf(t);
          y[q] = t;
        }
        y[0] += rv[4 * cb + g].x;
        y[1] += rv[4 * cb + g].y;
        y[2] += rv[4 * cb + g].z;
        y[3] += rv[4 * cb + g].w;
        const bool ok = mok && n < N;
        if (y_amax && ok)
          ymax = fmaxf(ymax, fmaxf(fmaxf(fabsf(y[0]), fabsf(y[1])), fmaxf(fabsf(y[2]), fabsf(y[3]))));
        const float4 yv = make_float4(y[0], y[1], y[2], y[3]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, yv), rY,
                                               ok ? ((unsigned)m * (unsigned)ldy + (unsigned)n) * 4u : OOB, 0, 0);
      }
    }
  }
  if (y_amax) sfx::publish_amax(ymax, y_amax, y_tag, s_wave);
}

template <int K>
void launch_narrow(const GemmArgs& a, hipStream_t st) {
  const int ncolblk = (a.N + NCOL - 1) / NCOL;
  const int ntiles = (a.M + 31) / 32;
  // two workgroups per CU (LDS 64 KB + registers), every column block of a row group on one XCD
  const int slots = 2 * 256;
  int nrowgrp = (ntiles + NRW - 1) / NRW;
  const int cap = slots / ncolblk > 0 ? slots / ncolblk : 1;
  if (nrowgrp > cap) nrowgrp = cap;
  int nb = ncolblk * nrowgrp;
  nb = (nb + 7) / 8 * 8;
  nrowgrp = nb / ncolblk;  // the padding rows groups find no tile (tile >= ntiles) and only stage W
  gemm_narrow_kernel<K><<<dim3((unsigned)nb), NRW * 64, 0, st>>>(
      a.M, a.N, a.A, a.lda, a.Wsp, a.winv, a.bias, a.act, a.act_ncols, a.R, a.ldr, a.Y, a.ldy, a.y_amax, a.y_tag,
      ncolblk, nrowgrp);
}

}  // namespace

namespace sfxg {

// SFX_GEMM_NARROW=0: these launches go to gemm_kernel as before
// (fp16x2 launches only: the caller checks split_mode(K) == 2, i.e. K >= 64 unless SFX_GEMM_PREC says otherwise)
bool gemm_narrow(const GemmArgs& a, int groups, bool vec, hipStream_t st) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("SFX_GEMM_NARROW");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!on || groups != 1 || !vec || !a.Wsp || !a.winv || a.gidx || a.pair_mode || a.out_rows || a.rowscale ||
      a.Ypre || a.scale || a.shift || a.dact || a.ridx || a.sk)
    return false;
  if (!(a.act == ACT_NONE || a.act == ACT_GELU)) return false;
  if (!(a.K == 64 || a.K == 96 || a.K == 128) || a.N % 4 != 0 || a.M < 1) return false;
  if (a.ldws != a.K || a.lda % 4 != 0 || a.ldy % 4 != 0 || (a.R && a.ldr % 4 != 0)) return false;
  if (!al16(a.A) || !al16(a.Y) || !al16(a.Wsp) || (a.R && !al16(a.R))) return false;
  // (an in-place residual, R == Y, is safe: every element is read and written by the same lane)
  if ((long long)a.M * a.lda * 4 + 64 >= (long long)OOB || (long long)a.M * a.ldy * 4 + 64 >= (long long)OOB ||
      (a.R && (long long)a.M * a.ldr * 4 + 64 >= (long long)OOB))
    return false;
  switch (a.K) {
    case 64: launch_narrow<64>(a, st); break;
    case 96: launch_narrow<96>(a, st); break;
    default: launch_narrow<128>(a, st); break;
  }
  return true;
}

}  // namespace sfxg
