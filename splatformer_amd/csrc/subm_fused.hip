// Block.cpe + shortcut + norm1 in one launch for C in {64, 96, 128} (reference calflops.py:45-53: x +=
// LN_cpe(Linear(SubMConv3d(x))); h = norm1(x); spconv SubMConv3d k=3, Pointcept Block.cpe -- SURVEY A.1.7):
//
//   x1 = x + LN_cpe(b' + sum_k sum_{nbr(i,k) = j} W'_k x_j),   h = LN1(x1)
//
// with the CPE Linear folded into the conv (W'_k = W_lin W_k, b' = W_lin b_conv + b_lin; ptv3.Block.cpe_fused).
// The offset-major pair GEMM (gemm.hip) writes one partial row per (offset, output) pair and a LayerNorm kernel
// reads them back; here the pair products never leave the chip:
//   * one workgroup owns SR = 128 consecutive output rows and their fp32 conv sums in LDS (initialised to b');
//   * for each offset k in ascending order, its rows with a neighbour are compacted (ballots, ascending row
//     order) into chunks of 16; a chunk's 16 gathered input rows are split into fp16x2 terms (per-row power-of-two
//     scale, sfx::split2h) in an LDS image shared by the 4 waves; each wave owns a fixed set of 16-column blocks
//     and holds W'_k of those columns as pre-split fp16x2 B fragments in registers (sfx_subm_cpe_pack); per block
//     h*h + h*l + l*h on v_mfma_f32_16x16x32_f16, fp32 accumulation; the 16 x 16 result is unscaled and added
//     to the LDS sums of its rows (a column block belongs to one wave: no races, and every row's sum is formed
//     in the same order -- bias, then k = 0..26 -- so results are bitwise reproducible);
//   * the epilogue runs LN_cpe, the shortcut and LN1 on the rows in LDS and writes x1 and h.
// HBM traffic per row: the gathered neighbour rows (mostly L2 hits), nbr, x, x1, h -- no centre output, no
// partial rows.  W'_k fragments are re-read from L2 per (workgroup, k): that re-read, not the MFMAs, bounds it.
#include "common.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int SR = 128;  // output rows per workgroup
constexpr int CHK = 16;  // compacted rows per chunk (the 16-row block of one 16x16x32 MFMA)

template <int C>
struct Cfg {
  static constexpr int NW = C <= 128 ? 4 : 8;     // waves per workgroup
  static constexpr int NTH = 64 * NW;
  static constexpr int NCB = C / 16;              // 16-column blocks
  static constexpr int NS = C / 32;               // 32-deep k-steps
  static constexpr int CBW = (NCB + NW - 1) / NW; // column blocks per wave (at most)
  static constexpr int SLOTS = C <= 64 ? 16 : (C <= 128 ? 32 : 64);  // float4 slots per gathered row (pow2 >= C/4)
  static constexpr int ACC_LD = C == 96 ? C : C + 4;  // floats per LDS sum row (C = 96: unpadded, 2 workgroups/CU)
  static constexpr int A_LD = 2 * C + 16;         // bytes per A-image row (one term)
  // LayerNorm epilogue: G lanes per row, NV float4 per lane
  static constexpr int G = C == 96 ? 8 : (C <= 128 ? C / 4 : 64);
  static constexpr int NV = C / (4 * G);
};

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// nn.LayerNorm over a row held by G lanes (float4 each, NV per lane): biased variance, two passes
template <int G, int NV>
__device__ __forceinline__ void ln_row4(const float4 (&v)[NV], const float* __restrict__ g,
                                        const float* __restrict__ b, float eps, int sub, float4 (&o)[NV]) {
  constexpr int C = 4 * G * NV;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = group_sum<G>(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float a = v[i].x - mean, bb = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
    q += (a * a + bb * bb) + (c * c + d * d);
  }
  const float rstd = 1.f / sqrtf(group_sum<G>(q) / (float)C + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * (sub + G * i);
    const float4 gg = *reinterpret_cast<const float4*>(g + c);
    const float4 bv = *reinterpret_cast<const float4*>(b + c);
    o[i] = make_float4((v[i].x - mean) * rstd * gg.x + bv.x, (v[i].y - mean) * rstd * gg.y + bv.y,
                       (v[i].z - mean) * rstd * gg.z + bv.z, (v[i].w - mean) * rstd * gg.w + bv.w);
  }
}

// power-of-two scale putting m in [2^14, 2^15) (1 for m == 0 or non-finite)
__device__ __forceinline__ float f16x2_scale(float m) {
  int e = 0;
  if (m > 0.f && m <= 3.4028235e38f) {
    (void)frexpf(m, &e);
    e = 15 - e;
    e = e > 126 ? 126 : (e < -126 ? -126 : e);
  }
  return ldexpf(1.f, e);
}

template <int C>
__global__ void __launch_bounds__(Cfg<C>::NTH, 2)
subm_cpe_ln_kernel(int n, const float* __restrict__ xc, const float* __restrict__ xres, const int* __restrict__ nbr,
                   const uint4* __restrict__ wpk, const float* __restrict__ winv, const float* __restrict__ bias,
                   const float* __restrict__ g_cpe, const float* __restrict__ b_cpe, const float* __restrict__ g1,
                   const float* __restrict__ b1, float eps, float* __restrict__ xout, float* __restrict__ hout) {
  using Q = Cfg<C>;
  constexpr int NG = CHK * Q::SLOTS / Q::NTH;  // gathered float4 slots per thread per chunk
  constexpr bool WDB = C <= 128;               // W'_k fragments double-buffered in registers (next offset prefetched)
  __shared__ __attribute__((aligned(16))) float acc[SR * Q::ACC_LD];
  __shared__ __attribute__((aligned(16))) unsigned char aimg[2][2][CHK * Q::A_LD];  // [buffer][term][row]
  __shared__ float ainv[2][CHK];          // 1 / (row scale) of a chunk's rows (0: padding row)
  __shared__ int lsrc[27][SR];            // per offset: compacted source rows
  __shared__ unsigned char lrow[27][SR];  // ... and the block rows they feed
  __shared__ int wcnt[27][2];
  __shared__ unsigned char item_k[27 * (SR / CHK)], item_c[27 * (SR / CHK)];  // flat chunk list
  __shared__ int s_nitems;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r0 = blockIdx.x * SR;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  for (int e = tid; e < SR * (C / 4); e += Q::NTH) {
    const int r = e / (C / 4), c4 = e - r * (C / 4);
    *reinterpret_cast<float4*>(&acc[r * Q::ACC_LD + 4 * c4]) = *reinterpret_cast<const float4*>(bias + 4 * c4);
  }
  // compaction of all 27 offsets: block rows with a neighbour at offset k, ascending (waves 0 and 1, a row each)
  int src[27], pos[27];
  if (tid < SR) {
    const int gi = r0 + tid;
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      src[k] = gi < n ? nbr[27ll * gi + k] : -1;
      const unsigned long long m = __ballot(src[k] >= 0);
      pos[k] = __popcll(m & lt_mask);
      if (lane == 0) wcnt[k][wid] = __popcll(m);
    }
  }
  __syncthreads();
  if (tid < SR) {
#pragma unroll
    for (int k = 0; k < 27; ++k)
      if (src[k] >= 0) {
        const int p = pos[k] + (wid == 1 ? wcnt[k][0] : 0);
        lsrc[k][p] = src[k];
        lrow[k][p] = (unsigned char)tid;
      }
  }
  if (tid == 0) {
    int ni = 0;
    for (int k = 0; k < 27; ++k) {
      const int nch = (wcnt[k][0] + wcnt[k][1] + CHK - 1) / CHK;
      for (int c = 0; c < nch; ++c, ++ni) {
        item_k[ni] = (unsigned char)k;
        item_c[ni] = (unsigned char)c;
      }
    }
    s_nitems = ni;
  }
  __syncthreads();
  const int nitems = s_nitems;

  // this wave's W'_k fragments [column block][k-step][term]; wn: the next offset's (prefetched, WDB)
  f16x8 wf[Q::CBW][Q::NS][2], wn[WDB ? Q::CBW : 1][Q::NS][2];
  auto load_w = [&](int k, f16x8 (&w)[Q::CBW][Q::NS][2]) {
#pragma unroll
    for (int i = 0; i < Q::CBW; ++i) {
      const int cb = wid + Q::NW * i;
      if (cb < Q::NCB) {
#pragma unroll
        for (int s = 0; s < Q::NS; ++s)
#pragma unroll
          for (int t = 0; t < 2; ++t)
            w[i][s][t] = __builtin_bit_cast(f16x8, wpk[((((long long)k * Q::NCB + cb) * Q::NS + s) * 2 + t) * 64 + lane]);
      }
    }
  };
  // next offset with chunks after item index c (27: none)
  auto next_k = [&](int c) {
    const int k = item_k[c];
    for (int j = c + 1; j < nitems; ++j)
      if (item_k[j] != k) return (int)item_k[j];
    return 27;
  };
  // chunk gather: this thread's NG float4 slots of item c's 16 rows
  auto gather = [&](int c, float4 (&v)[NG]) {
    const int k = item_k[c], cnt = wcnt[k][0] + wcnt[k][1];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int e = tid + Q::NTH * g;
      const int row = e / Q::SLOTS, slot = e - row * Q::SLOTS;
      const int p = item_c[c] * CHK + row;
      v[g] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p < cnt && slot < C / 4) v[g] = *reinterpret_cast<const float4*>(xc + (long long)lsrc[k][p] * C + 4 * slot);
    }
  };
  // split the gathered rows into chunk image b (per-row power-of-two scale)
  auto stage = [&](int c, int b, const float4 (&v)[NG]) {
    const int k = item_k[c], cnt = wcnt[k][0] + wcnt[k][1];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int e = tid + Q::NTH * g;
      const int row = e / Q::SLOTS, slot = e - row * Q::SLOTS;
      const int p = item_c[c] * CHK + row;
      float m = fmaxf(fmaxf(fabsf(v[g].x), fabsf(v[g].y)), fmaxf(fabsf(v[g].z), fabsf(v[g].w)));
#pragma unroll
      for (int o = Q::SLOTS / 2; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      const float sc = f16x2_scale(m);
      if (slot < C / 4) {
        uint2 t[2];
        sfx::split2h(v[g], sc, t);
        *reinterpret_cast<uint2*>(&aimg[b][0][row * Q::A_LD + 8 * slot]) = t[0];
        *reinterpret_cast<uint2*>(&aimg[b][1][row * Q::A_LD + 8 * slot]) = t[1];
      }
      if (slot == 0) ainv[b][row] = p < cnt ? 1.f / sc : 0.f;
    }
  };

  if (nitems > 0) {
    float4 v[NG];
    load_w(item_k[0], wf);
    gather(0, v);
    if constexpr (WDB) {
      const int k1 = next_k(0);
      if (k1 < 27) load_w(k1, wn);
    }
    stage(0, 0, v);
  }
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < nitems; ++c) {
    const int b = c & 1;
    const int k = item_k[c], cnt = wcnt[k][0] + wcnt[k][1];
    float4 v[NG];
    if (c + 1 < nitems) gather(c + 1, v);  // next chunk's rows: in flight during this chunk's MFMAs
    f16x8 af[Q::NS][2];  // this chunk's A fragments (rows lane & 15, k = 32 s + 8 (lane >> 4) ..)
#pragma unroll
    for (int s = 0; s < Q::NS; ++s) {
      const int off = (lane & 15) * Q::A_LD + (32 * s + 8 * (lane >> 4)) * 2;
      af[s][0] = *reinterpret_cast<const f16x8*>(&aimg[b][0][off]);
      af[s][1] = *reinterpret_cast<const f16x8*>(&aimg[b][1][off]);
    }
    float rinv[4];
    int rrow[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 4 * (lane >> 4) + q;
      const int p = item_c[c] * CHK + row;
      rinv[q] = ainv[b][row];
      rrow[q] = p < cnt ? (int)lrow[k][p] : -1;
    }
#pragma unroll
    for (int i = 0; i < Q::CBW; ++i) {
      const int cb = wid + Q::NW * i;
      if (cb < Q::NCB) {
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < Q::NS; ++s) {
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[s][1], wf[i][s][0], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[s][0], wf[i][s][1], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[s][0], wf[i][s][0], d, 0, 0, 0);
        }
        const int o = 16 * cb + (lane & 15);
        const float wi = winv[o];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (rrow[q] >= 0) {
            float* a = &acc[rrow[q] * Q::ACC_LD + o];
            *a += d[q] * rinv[q] * wi;
          }
        }
      }
    }
    if (c + 1 < nitems) {
      stage(c + 1, b ^ 1, v);
      const int kn = item_k[c + 1];
      if (kn != k) {  // the next chunk starts a new offset
        if constexpr (WDB) {
#pragma unroll
          for (int i = 0; i < Q::CBW; ++i)
#pragma unroll
            for (int s = 0; s < Q::NS; ++s) {
              wf[i][s][0] = wn[i][s][0];
              wf[i][s][1] = wn[i][s][1];
            }
          const int k2 = next_k(c + 1);
          if (k2 < 27) load_w(k2, wn);
        } else {
          load_w(kn, wf);
        }
      }
    }
    __syncthreads();
  }

  // epilogue: LN_cpe -> + shortcut -> LN1, G lanes per row
  constexpr int G = Q::G, NV = Q::NV;
  const int sub = tid % G;
#pragma unroll 1
  for (int rb = 0; rb < SR; rb += Q::NTH / G) {
    const int row = rb + tid / G;
    const int gi = r0 + row;
    const bool ok = gi < n;
    float4 v[NV], o[NV], x[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = 4 * (sub + G * i);
      v[i] = *reinterpret_cast<const float4*>(&acc[row * Q::ACC_LD + c]);
      x[i] = ok ? *reinterpret_cast<const float4*>(xres + (long long)gi * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    ln_row4<G, NV>(v, g_cpe, b_cpe, eps, sub, o);
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = make_float4(x[i].x + o[i].x, x[i].y + o[i].y, x[i].z + o[i].z, x[i].w + o[i].w);
    ln_row4<G, NV>(v, g1, b1, eps, sub, o);
    if (ok) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = 4 * (sub + G * i);
        *reinterpret_cast<float4*>(xout + (long long)gi * C + c) = v[i];
        *reinterpret_cast<float4*>(hout + (long long)gi * C + c) = o[i];
      }
    }
  }
}

// per output column o of W' [C, 27 C]: the fp16x2 scale of the whole column (max over every offset and input)
__global__ void __launch_bounds__(64) subm_cpe_wscale_kernel(int C, const float* __restrict__ w,
                                                             float* __restrict__ winv, float* __restrict__ wsc) {
  const int o = blockIdx.x;
  float m = 0.f;
  for (int e = threadIdx.x; e < 27 * C; e += 64) m = fmaxf(m, fabsf(w[(long long)o * 27 * C + e]));
  m = sfx::wave_max(m);
  if (threadIdx.x == 0) {
    const float s = f16x2_scale(m);
    wsc[o] = s;
    winv[o] = 1.f / s;
  }
}

// fragments: [k][column block][k-step][term][lane] x 8 halves; lane l holds B[in = 32s + 8(l>>4) + j][o = 16cb + (l&15)]
__global__ void subm_cpe_pack_kernel(int C, const float* __restrict__ w, const float* __restrict__ wsc,
                                     uint4* __restrict__ wpk) {
  const int NCB = C / 16, NS = C / 32;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // (k, cb, s, lane)
  const long long total = 27ll * NCB * NS * 64;
  if (t >= total) return;
  const int lane = (int)(t & 63);
  long long q = t >> 6;
  const int s = (int)(q % NS);
  q /= NS;
  const int cb = (int)(q % NCB);
  const int k = (int)(q / NCB);
  const int o = 16 * cb + (lane & 15);
  const int in0 = 32 * s + 8 * (lane >> 4);
  const float* src = w + (long long)o * 27 * C + (long long)k * C + in0;
  const float sc = wsc[o];
  uint2 a[2], b[2];
  sfx::split2h(make_float4(src[0], src[1], src[2], src[3]), sc, a);
  sfx::split2h(make_float4(src[4], src[5], src[6], src[7]), sc, b);
  const long long f = (((long long)k * NCB + cb) * NS + s) * 2;
  wpk[f * 64 + lane] = make_uint4(a[0].x, a[0].y, b[0].x, b[0].y);
  wpk[(f + 1) * 64 + lane] = make_uint4(a[1].x, a[1].y, b[1].x, b[1].y);
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

// bytes of the packed fp16x2 conv weight of sfx_subm_cpe_ln (0: C not served)
size_t sfx_subm_cpe_pack_bytes(int C) {
  if (C != 64 && C != 96 && C != 128) return 0;
  return (size_t)27 * C * C * 4;
}

// W' [C, 27*C] (row o = output channel, column k*C + i: the spconv [Cout, 3, 3, 3, Cin] layout with the CPE
// Linear folded in) -> packed fragments (sfx_subm_cpe_pack_bytes(C)) + inverse column scales winv[C]
// (ws: C floats of scratch)
int sfx_subm_cpe_pack(int C, const float* w, void* wpk, float* winv, float* ws, void* stream) {
  SFX_REQUIRE(sfx_subm_cpe_pack_bytes(C) > 0, "sfx_subm_cpe_pack: C must be 64, 96 or 128");
  SFX_REQUIRE(w && wpk && winv && ws, "sfx_subm_cpe_pack: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  subm_cpe_wscale_kernel<<<C, 64, 0, st>>>(C, w, winv, ws);
  const long long total = 27ll * (C / 16) * (C / 32) * 64;
  subm_cpe_pack_kernel<<<sfx::ceil_div(total, 256), 256, 0, st>>>(C, w, ws, reinterpret_cast<uint4*>(wpk));
  return sfx::check_launch("sfx_subm_cpe_pack");
}

// x1 = xres + LN_cpe(bias + SubMConv(xc)), h = LN1(x1) (see the top of this file); rows contiguous [n, C]
int sfx_subm_cpe_ln(int n, int C, const float* xc, const float* xres, const int* nbr, const void* wpk,
                    const float* winv, const float* bias, const float* gamma_cpe, const float* beta_cpe,
                    const float* gamma1, const float* beta1, float eps, float* x_out, float* h_out, void* stream) {
  SFX_REQUIRE(n >= 0 && sfx_subm_cpe_pack_bytes(C) > 0, "sfx_subm_cpe_ln: C must be 64, 96 or 128");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(xc && xres && nbr && wpk && winv && bias && gamma_cpe && beta_cpe && gamma1 && beta1 && x_out && h_out,
              "sfx_subm_cpe_ln: null buffer");
  SFX_REQUIRE(al16(xc) && al16(xres) && al16(wpk) && al16(bias) && al16(gamma_cpe) && al16(beta_cpe) &&
                  al16(gamma1) && al16(beta1) && al16(x_out) && al16(h_out),
              "sfx_subm_cpe_ln: buffers must be 16-byte aligned");
  hipStream_t st = sfx::as_stream(stream);
  const unsigned grid = sfx::ceil_div(n, SR);
  const uint4* wp = reinterpret_cast<const uint4*>(wpk);
#define SFX_SUBM_LN(CC)                                                                                         \
  subm_cpe_ln_kernel<CC><<<grid, Cfg<CC>::NTH, 0, st>>>(n, xc, xres, nbr, wp, winv, bias, gamma_cpe, beta_cpe, gamma1, \
                                                         beta1, eps, x_out, h_out)
  if (C == 64) SFX_SUBM_LN(64);
  else if (C == 96) SFX_SUBM_LN(96);
  else SFX_SUBM_LN(128);
#undef SFX_SUBM_LN
  return sfx::check_launch("sfx_subm_cpe_ln");
}

}  // extern "C"
