// Serialized windowed multi-head attention (PTv3 SerializedAttention,
// non-flash path: reference models/pointtransformer_v3.py:121-126 patch 128,
// math restated in-tree at visualize.py:140-179).
//
// For each window of K <= 128 consecutive serialized positions and each head:
//   S = (q * scale) k^T ; P = softmax_keys(S) ; O = P v
// q/k/v rows are gathered straight from the qkv projection [N, 3C] through
// the serialized order (`qkv[order]`, row layout [3][H][d]) and the output row
// is scattered back through the same order (`feat[inverse]`), so neither the
// padded/permuted qkv nor the [N', H, K, K] score tensor is materialised.
//
// Window table: win[w] = (key_start, query_start) in serialized positions.
// Pointcept pads a ragged last window by duplicating the K - n%K points that
// precede it (get_padding_and_inverse); that window therefore attends over
// the last K real points and only its new queries are written -- the table
// encodes exactly that (key_start = n - K, query_start = floor(n/K)*K).
//
// gfx950: one 256-thread workgroup per (window, head), 4 waves x 32 queries.
// S^T = K Q^T on v_mfma_f32_32x32x2_f32 puts each query on a lane column and
// its 128 keys in registers (64 per half-wave), so the softmax is a register
// reduction + one cross-half exchange, and P^T feeds the P.V MFMA directly as
// the B operand (no LDS round trip for P).
#include <cstdlib>

#include <type_traits>

#include "common.h"

extern "C" int sfx_get_precision(void);  // gemm.hip (include/sfx.h)

#ifndef SFX_ATTN_OCC16
#define SFX_ATTN_OCC16 4  // workgroups per CU the d = 16 split kernel is compiled for
#endif

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int KMAX = 128;

// V^T chunk swizzle: the 16-byte chunk c (8 keys) of V^T row dd sits at chunk c ^ vt_swz(dd), 2 x the parity of
// dd's 4-row group.  The staging's transposed dword stores (rows 4 ch .. 4 ch + 3 of 4-8 column chunks per 32
// lanes) were 2- / 3- / 4-way bank conflicts at d = 16 / 24 / 32 (the stride-136 rows put every other chunk group on
// one bank set); swizzled they are 1- / 2- / 2-way (free for ds_write_b32), and the fragment reads stay conflict-
// free (tools/attn_banks.py)
__device__ __forceinline__ int vt_swz(int dd) { return (__builtin_popcount((unsigned)(dd >> 2)) & 1) << 1; }

template <int D>
__global__ void __launch_bounds__(256, 2)
window_attn_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win,
                   int Kwin, int C, float scale, float* __restrict__ out) {
  constexpr int DP = D + 4;   // Q/K rows: conflict-free ds_read_b128 for D = 16, 24, 32
  constexpr int DPV = 40;     // V rows padded to 32 (+8): the P.V MFMA reads V^T[dd = lane][key] with no
                              // masking for dd >= D, and the two half-waves (keys 4 apart) hit disjoint banks
  constexpr int HALF = D / 2;  // k-values per lane half in S = K Q^T
  __shared__ __attribute__((aligned(16))) float Qs[KMAX * DP];
  __shared__ __attribute__((aligned(16))) float Ks[KMAX * DP];
  __shared__ __attribute__((aligned(16))) float Vs[KMAX * DPV];
  __shared__ int rows[KMAX];

  const int w = blockIdx.x, head = blockIdx.y;
  const int key_start = win[2 * w], query_start = win[2 * w + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  if (tid < KMAX) rows[tid] = tid < Kwin ? order[key_start + tid] : -1;
  if (D < 32)  // zero the V padding columns D..31 once
    for (int e = tid; e < KMAX * (32 - D) / 4; e += 256) {
      const int row = e / ((32 - D) / 4), c4 = e - row * ((32 - D) / 4);
      *reinterpret_cast<float4*>(&Vs[row * DPV + D + 4 * c4]) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  __syncthreads();
  // gather q/k/v rows of this head: KMAX rows x 3 mats x D/4 float4
  constexpr int CH = D / 4;
  for (int e = tid; e < KMAX * 3 * CH; e += 256) {
    const int row = e / (3 * CH);
    const int rem = e - row * 3 * CH;
    const int mat = rem / CH, ch = rem - mat * CH;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int src = rows[row];
    if (src >= 0) v = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + mat * C + head * D + 4 * ch);
    if (mat == 0) {
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      *reinterpret_cast<float4*>(&Qs[row * DP + 4 * ch]) = v;
    } else if (mat == 1) {
      *reinterpret_cast<float4*>(&Ks[row * DP + 4 * ch]) = v;
    } else {
      *reinterpret_cast<float4*>(&Vs[row * DPV + 4 * ch]) = v;
    }
  }
  __syncthreads();

  // S^T[key][query] for this wave's 32 queries, 4 key blocks of 32
  floatx16 s[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
  const float* qrow = &Qs[(32 * wid + l32) * DP + h * HALF];
#pragma unroll
  for (int c = 0; c < HALF / 4; ++c) {
    const float4 qv = *reinterpret_cast<const float4*>(qrow + 4 * c);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const float4 kv = *reinterpret_cast<const float4*>(&Ks[(kb * 32 + l32) * DP + h * HALF + 4 * c]);
      s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qv.x, s[kb], 0, 0, 0);
      s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qv.y, s[kb], 0, 0, 0);
      s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qv.z, s[kb], 0, 0, 0);
      s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qv.w, s[kb], 0, 0, 0);
    }
  }
  // softmax over keys (register axis + the other half-wave); keys >= Kwin only exist in short windows
  if (Kwin < KMAX) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (key >= Kwin) s[kb][r] = -INFINITY;
      }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = __expf(s[kb][r] - mx);
      s[kb][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float rinv = 1.f / sum;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] *= rinv;

  // O^T[dd][query] = sum_key V[key][dd] P^T[key][query]
  floatx16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  const float* vcol = &Vs[4 * h * DPV + l32];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int key0 = kb * 32 + (st & 3) + 8 * (st >> 2);  // + 4h folded into vcol
      o = __builtin_amdgcn_mfma_f32_32x32x2f32(vcol[key0 * DPV], s[kb][st], o, 0, 0, 0);
    }

  // scatter: query 32*wid + l32 (lane column), dd rows (r&3) + 8(r>>2) + 4h
  const int qi = 32 * wid + l32;
  const int qpos = key_start + qi;
  if (qi < Kwin && qpos >= query_start) {
    float* dst = out + (long long)rows[qi] * C + head * D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dd = 8 * g + 4 * h;
      if (dd + 3 < D) {
        *reinterpret_cast<float4*>(dst + dd) = make_float4(o[4 * g + 0], o[4 * g + 1], o[4 * g + 2], o[4 * g + 3]);
      }
    }
  }
}

// ---- flash mode: windows of up to 2^20 keys, per-window key count -------------------------------------
// Reference pointtransformer_v3.py:121-123 (patch 1024 when enable_flash) and Pointcept's SerializedAttention
// flash branch: the padded serialized sequence is cut at cu_seqlens, so a batch of n <= K points is ONE window
// of n keys (no padding) and a longer batch has windows of K keys, its ragged last one padded with the points
// that precede it (the same (key_start, query_start) encoding as above).  Table win3[w] = (key_start,
// query_start, key_count).
//
// One 256-thread workgroup per (window, 128-query block, head): the 128 queries stay in registers as S^T
// columns while the window's keys stream through LDS in 128-key blocks with an online softmax (running max and
// sum per query, accumulator rescaled by exp(m_old - m_new)), exact fp32 MFMA (v_mfma_f32_32x32x2_f32) --
// the same S^T = K Q^T / O^T = V^T P^T register dataflow as window_attn_kernel, K/V LDS images reused per
// block.  Query blocks past the window's count or wholly before its query_start exit before any barrier.
template <int D>
__global__ void __launch_bounds__(256, 2)
window_attn_flash_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win3,
                         int qblocks, int C, float scale, float* __restrict__ out) {
  constexpr int DP = D + 4;
  constexpr int DPV = 40;
  constexpr int HALF = D / 2;
  constexpr int CH = D / 4;
  __shared__ __attribute__((aligned(16))) float Qs[KMAX * DP];
  __shared__ __attribute__((aligned(16))) float Ks[KMAX * DP];
  __shared__ __attribute__((aligned(16))) float Vs[KMAX * DPV];
  __shared__ int qrows[KMAX];
  __shared__ int krows[KMAX];

  const int w = blockIdx.x / qblocks, qb = blockIdx.x - w * qblocks, head = blockIdx.y;
  const int key_start = win3[3 * w], query_start = win3[3 * w + 1], count = win3[3 * w + 2];
  const int q0 = qb * KMAX;  // window-relative first query of this block
  if (q0 >= count || key_start + q0 + KMAX <= query_start) return;  // workgroup-uniform, before any barrier
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  if (tid < KMAX) qrows[tid] = q0 + tid < count ? order[key_start + q0 + tid] : -1;
  if (D < 32)
    for (int e = tid; e < KMAX * (32 - D) / 4; e += 256) {
      const int row = e / ((32 - D) / 4), c4 = e - row * ((32 - D) / 4);
      *reinterpret_cast<float4*>(&Vs[row * DPV + D + 4 * c4]) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  __syncthreads();
  for (int e = tid; e < KMAX * CH; e += 256) {
    const int row = e / CH, ch = e - row * CH;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int src = qrows[row];
    if (src >= 0) v = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + head * D + 4 * ch);
    v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    *reinterpret_cast<float4*>(&Qs[row * DP + 4 * ch]) = v;
  }
  __syncthreads();
  float4 qv[HALF / 4];
#pragma unroll
  for (int c = 0; c < HALF / 4; ++c)
    qv[c] = *reinterpret_cast<const float4*>(&Qs[(32 * wid + l32) * DP + h * HALF + 4 * c]);

  float m_run = -INFINITY, l_run = 0.f;
  floatx16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  const float* vcol = &Vs[4 * h * DPV + l32];

  for (int k0 = 0; k0 < count; k0 += KMAX) {
    const int nk = min(KMAX, count - k0);
    __syncthreads();  // the previous block's K/V fragment reads are done
    if (tid < KMAX) krows[tid] = tid < nk ? order[key_start + k0 + tid] : -1;
    __syncthreads();
    for (int e = tid; e < KMAX * 2 * CH; e += 256) {
      const int row = e / (2 * CH);
      const int rem = e - row * 2 * CH;
      const int mat = rem / CH, ch = rem - mat * CH;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int src = krows[row];
      if (src >= 0) v = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + (mat + 1) * C + head * D + 4 * ch);
      if (mat == 0) *reinterpret_cast<float4*>(&Ks[row * DP + 4 * ch]) = v;
      else *reinterpret_cast<float4*>(&Vs[row * DPV + 4 * ch]) = v;
    }
    __syncthreads();

    floatx16 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
    for (int c = 0; c < HALF / 4; ++c) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float4 kv = *reinterpret_cast<const float4*>(&Ks[(kb * 32 + l32) * DP + h * HALF + 4 * c]);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qv[c].x, s[kb], 0, 0, 0);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qv[c].y, s[kb], 0, 0, 0);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qv[c].z, s[kb], 0, 0, 0);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qv[c].w, s[kb], 0, 0, 0);
      }
    }
    if (nk < KMAX) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (key >= nk) s[kb][r] = -INFINITY;
        }
    }
    float bm = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) bm = fmaxf(bm, s[kb][r]);
    bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
    const float m_new = fmaxf(m_run, bm);  // finite: every block holds at least one key
    const float corr = __expf(m_run - m_new);
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __expf(s[kb][r] - m_new);
        s[kb][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 32, 64);
    l_run = l_run * corr + sum;
    m_run = m_new;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] *= corr;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int key0 = kb * 32 + (st & 3) + 8 * (st >> 2);
        o = __builtin_amdgcn_mfma_f32_32x32x2f32(vcol[key0 * DPV], s[kb][st], o, 0, 0, 0);
      }
  }

  const float rinv = 1.f / l_run;
  const int qi = q0 + 32 * wid + l32;
  if (qi < count && key_start + qi >= query_start) {
    float* dst = out + (long long)qrows[32 * wid + l32] * C + head * D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dd = 8 * g + 4 * h;
      if (dd + 3 < D)
        *reinterpret_cast<float4*>(dst + dd) = make_float4(o[4 * g + 0] * rinv, o[4 * g + 1] * rinv,
                                                           o[4 * g + 2] * rinv, o[4 * g + 3] * rinv);
    }
  }
}

// ---- flash mode backward (training with enable_flash=True) ----------------------------------------------
// Two launches, fp32 VALU (each lane owns one query or one key; the block's other rows stream through LDS as
// wave-wide broadcasts):
//   query pass: per query i of window w (i >= query_start): m_i, l_i and O_i (online softmax over the window's
//     keys), lse_i = m_i + log l_i, delta_i = dO_i . O_i / l_i, then dQ_i = scale sum_j P_ij (dO_i.v_j - delta_i)
//     k_j (plain store: a point is a query of exactly one window); (lse, delta) saved per (point, head).
//   key pass: per key j of window w: dV_j += sum_i P_ij dO_i, dK_j += scale sum_i P_ij (dO_i.v_j - delta_i) q_i
//     over the window's own queries; float atomics into dqkv (the keys of a ragged last window are also keys of
//     the window before it: two adds onto the zero-filled buffer, order-independent).
constexpr int FB = 128;  // rows per workgroup and per LDS block

template <int D>
__global__ void __launch_bounds__(FB)
flash_bwd_query_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win3,
                       int qblocks, int C, int H, float scale, const float* __restrict__ dout,
                       float* __restrict__ dqkv, float* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) float Ks[FB * D];
  __shared__ __attribute__((aligned(16))) float Vs[FB * D];
  __shared__ int krows[FB];
  const int w = blockIdx.x / qblocks, qb = blockIdx.x - w * qblocks, head = blockIdx.y;
  const int ks = win3[3 * w], qs = win3[3 * w + 1], cnt = win3[3 * w + 2];
  const int q0 = qb * FB;
  if (q0 >= cnt || ks + q0 + FB <= qs) return;  // workgroup-uniform, before any barrier
  const int t = threadIdx.x, qi = q0 + t;
  const bool valid = qi < cnt && ks + qi >= qs;
  const int row = valid ? order[ks + qi] : 0;
  const long long ld = 3ll * C;
  float q[D], g[D], o[D], dq[D];
#pragma unroll
  for (int c = 0; c < D; ++c) {
    q[c] = valid ? qkv[(long long)row * ld + head * D + c] * scale : 0.f;
    g[c] = valid ? dout[(long long)row * C + head * D + c] : 0.f;
    o[c] = 0.f;
    dq[c] = 0.f;
  }
  auto stage = [&](int k0, int nk) {
    __syncthreads();
    krows[t] = t < nk ? order[ks + k0 + t] : -1;
    __syncthreads();
    for (int e = t; e < FB * D / 4; e += FB) {
      const int r = e / (D / 4), c4 = e - r * (D / 4);
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
      if (krows[r] >= 0) {
        const float* src = qkv + (long long)krows[r] * ld + head * D + 4 * c4;
        kv = *reinterpret_cast<const float4*>(src + C);
        vv = *reinterpret_cast<const float4*>(src + 2 * C);
      }
      *reinterpret_cast<float4*>(&Ks[r * D + 4 * c4]) = kv;
      *reinterpret_cast<float4*>(&Vs[r * D + 4 * c4]) = vv;
    }
    __syncthreads();
  };
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < cnt; k0 += FB) {
    const int nk = min(FB, cnt - k0);
    stage(k0, nk);
    for (int j = 0; j < nk; ++j) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < D; ++c) s = fmaf(q[c], Ks[j * D + c], s);
      const float mn = fmaxf(m, s);
      const float corr = expf(m - mn), p = expf(s - mn);
      l = l * corr + p;
#pragma unroll
      for (int c = 0; c < D; ++c) o[c] = fmaf(p, Vs[j * D + c], o[c] * corr);
      m = mn;
    }
  }
  float delta = 0.f;
#pragma unroll
  for (int c = 0; c < D; ++c) delta = fmaf(g[c], o[c], delta);
  delta /= l;
  const float lse = m + logf(l);
  for (int k0 = 0; k0 < cnt; k0 += FB) {
    const int nk = min(FB, cnt - k0);
    stage(k0, nk);
    for (int j = 0; j < nk; ++j) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        s = fmaf(q[c], Ks[j * D + c], s);
        dp = fmaf(g[c], Vs[j * D + c], dp);
      }
      const float ds = expf(s - lse) * (dp - delta);
#pragma unroll
      for (int c = 0; c < D; ++c) dq[c] = fmaf(ds, Ks[j * D + c], dq[c]);
    }
  }
  if (valid) {
#pragma unroll
    for (int c = 0; c < D; ++c) dqkv[(long long)row * ld + head * D + c] = dq[c] * scale;
    stats[((long long)row * H + head) * 2] = lse;
    stats[((long long)row * H + head) * 2 + 1] = delta;
  }
}

template <int D>
__global__ void __launch_bounds__(FB)
flash_bwd_key_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win3,
                     int kblocks, int C, int H, float scale, const float* __restrict__ dout,
                     float* __restrict__ dqkv, const float* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) float Qs[FB * D];
  __shared__ __attribute__((aligned(16))) float Gs[FB * D];
  __shared__ float Ls[FB], Ds[FB];
  __shared__ int qrows[FB];
  const int w = blockIdx.x / kblocks, kb = blockIdx.x - w * kblocks, head = blockIdx.y;
  const int ks = win3[3 * w], qs = win3[3 * w + 1], cnt = win3[3 * w + 2];
  const int k0 = kb * FB;
  if (k0 >= cnt) return;  // workgroup-uniform
  const int t = threadIdx.x, kj = k0 + t;
  const bool valid = kj < cnt;
  const int row = valid ? order[ks + kj] : 0;
  const long long ld = 3ll * C;
  float k[D], v[D], dk[D], dv[D];
#pragma unroll
  for (int c = 0; c < D; ++c) {
    k[c] = valid ? qkv[(long long)row * ld + C + head * D + c] : 0.f;
    v[c] = valid ? qkv[(long long)row * ld + 2 * C + head * D + c] : 0.f;
    dk[c] = 0.f;
    dv[c] = 0.f;
  }
  for (int i0 = qs - ks; i0 < cnt; i0 += FB) {  // the window's own queries
    const int ni = min(FB, cnt - i0);
    __syncthreads();
    qrows[t] = t < ni ? order[ks + i0 + t] : -1;
    __syncthreads();
    for (int e = t; e < FB * D / 4; e += FB) {
      const int r = e / (D / 4), c4 = e - r * (D / 4);
      float4 qv = make_float4(0.f, 0.f, 0.f, 0.f), gv = qv;
      if (qrows[r] >= 0) {
        qv = *reinterpret_cast<const float4*>(qkv + (long long)qrows[r] * ld + head * D + 4 * c4);
        qv.x *= scale; qv.y *= scale; qv.z *= scale; qv.w *= scale;
        gv = *reinterpret_cast<const float4*>(dout + (long long)qrows[r] * C + head * D + 4 * c4);
      }
      *reinterpret_cast<float4*>(&Qs[r * D + 4 * c4]) = qv;
      *reinterpret_cast<float4*>(&Gs[r * D + 4 * c4]) = gv;
    }
    Ls[t] = t < ni ? stats[((long long)qrows[t] * H + head) * 2] : INFINITY;
    Ds[t] = t < ni ? stats[((long long)qrows[t] * H + head) * 2 + 1] : 0.f;
    __syncthreads();
    for (int i = 0; i < ni; ++i) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        s = fmaf(Qs[i * D + c], k[c], s);
        dp = fmaf(Gs[i * D + c], v[c], dp);
      }
      const float p = expf(s - Ls[i]);
      const float ds = p * (dp - Ds[i]);
#pragma unroll
      for (int c = 0; c < D; ++c) {
        dv[c] = fmaf(p, Gs[i * D + c], dv[c]);
        dk[c] = fmaf(ds, Qs[i * D + c], dk[c]);
      }
    }
  }
  if (valid) {
    float* dst = dqkv + (long long)row * ld + head * D;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      atomicAdd(dst + C + c, dk[c]);
      atomicAdd(dst + 2 * C + c, dv[c]);
    }
  }
}

// ---- split-bf16 forward (default) ---------------------------------------------------------------------
// The same dataflow on v_mfma_f32_32x32x16_bf16: q, k, v and p enter as three bf16 terms each
// (sfx::split3) and every 32x32x16 block is the six leading term products accumulated in fp32 -- fp32
// accuracy at 6 x 32 MFMA cycles per 16-deep step instead of 8 x 64 on v_mfma_f32_32x32x2_f32.
//   S^T = K Q^T: A = K [key][dd], B = Q^T, KD = 16 (D = 16) or 32 (D = 24, 32; columns >= D zero).
//   O^T = V^T P^T: B = P^T straight from the softmax registers -- registers 8s..8s+7 of key block kb are
//   the 16-key step s (element j <-> key 32kb + 16s + 8(j>>2) + 4h + (j&3)); A = V^T, staged transposed
//   with the keys of every 16-key group permuted to that order so a lane's 8 keys are one 16-byte read.
// LDS: K term image [3][128][KD] (KD = 16: 48-byte rows; KD = 32: 64-byte rows, 16-byte chunks XOR-
// swizzled by row >> 2), V^T [3][D][136] (272-byte rows; lanes dd >= D feed zero fragments); all fragment
// reads are conflict-free.  Q never touches LDS: each lane gathers and splits its own query's 8-wide
// slices.  31-50 KB per workgroup: 3-4 workgroups per CU to hide the row gathers.
//
// F16 (when the caller passes an amax slot bounding |qkv|): fp16x2 terms instead -- q, k, v scaled by a
// power of two that puts the bound in [2^14, 2^15), the unnormalised probabilities (0, 1] by 2^14, two fp16
// terms each (sfx::split2h), three term products per block on v_mfma_f32_32x32x16_f16; S and O are unscaled
// in registers.  Same fp32-level accuracy, half the MFMAs and two-thirds of the LDS images.
// ONE (sfx_set_precision(1), the reference's autocast class): F16 the leading product h*h only, bf16x3 the three
// leading term products (16-bit significands)
template <int D, bool F16, bool ONE = false>
__global__ void __launch_bounds__(256, D == 16 ? SFX_ATTN_OCC16 : 3)
window_attn_split_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win,
                         int Kwin, int C, float scale, float* __restrict__ out,
                         const unsigned long long* __restrict__ qkv_amax, unsigned qkv_tag, int nwin) {
  typedef typename std::conditional<F16, _Float16, __bf16>::type elem_t;
  typedef elem_t bf16x8 __attribute__((ext_vector_type(8)));  // (fragment type: bf16 or fp16 terms)
  constexpr int NT = F16 ? 2 : 3;            // terms per operand
  constexpr int KD = D == 16 ? 16 : 32;
  constexpr int NKS = KD / 16;
  constexpr int QROW = KD == 16 ? 48 : 64;  // bytes per Q/K term row
  constexpr int VST = 136;                  // V^T row stride (16-bit elements)
  constexpr int QK_BYTES = NT * KMAX * QROW;
  constexpr int V_BYTES = NT * D * VST * 2;
  // operand scales (F16): qkv by sq, probabilities by 2^14
  float sq = 1.f, iq = 1.f;
  if constexpr (F16) {
    const float m = sfx::read_amax(qkv_amax, qkv_tag);
    int e = 0;
    if (m > 0.f && m <= 3.4028235e38f) {
      (void)frexpf(m, &e);
      e = 15 - e;
      e = e > 126 ? 126 : (e < -126 ? -126 : e);
    }
    sq = ldexpf(1.f, e);
    iq = ldexpf(1.f, -e);
  }
  auto split = [&](float4 v, float sc, uint2 (&t)[NT]) {
    if constexpr (F16) sfx::split2h(v, sc, t); else sfx::split3(v, t);
  };
  __shared__ __attribute__((aligned(16))) char lds[QK_BYTES + V_BYTES];
  __shared__ int rows[KMAX];
  char* Ks = lds;
  unsigned short* Vt = reinterpret_cast<unsigned short*>(lds + QK_BYTES);
  // byte offset of 16-byte chunk c of term row r
  auto qk_off = [](int r, int c) -> int {
    return KD == 16 ? r * 48 + c * 16 : r * 64 + (((c ^ (r >> 2)) & 3) << 4);
  };

  // XCD-aware numbering over a 1-D grid padded to a multiple of 8: consecutive blocks go round-robin to the 8
  // XCDs, so logical id L = xcd * (grid / 8) + slot puts all heads of a window on one XCD back to back -- the
  // 128-byte qkv lines its heads share (d = 16: two heads per line) are fetched from HBM once into that L2.
  const int heads = C / D;
  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8);
  if (L >= nwin * heads) return;
  const int w = L / heads, head = L - w * heads;
  const int key_start = win[2 * w], query_start = win[2 * w + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  if (tid < KMAX) rows[tid] = tid < Kwin ? order[key_start + tid] : -1;
  // zero padding: K columns D..KD-1 (never written by the staging below)
  if (D < KD)
    for (int rr = tid; rr < NT * KMAX; rr += 256)  // term rows, term-major
      *reinterpret_cast<uint4*>(Ks + qk_off(rr, D / 8)) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  // gather + split, one matrix at a time (wave-uniform paths): q, k rows as KMAX x D/4 float4; v as
  // key pairs x D/4 float4 so the transposed V^T writes are whole dwords (keys 2m, 2m+1 are adjacent
  // in the permuted order)
  constexpr int CH = D / 4;
  typedef unsigned uintx4 __attribute__((ext_vector_type(4)));
  // this lane's query slices (B operand of S^T = K Q^T): dd = 16 ks + 8h + j, zero past D
  bf16x8 qf[NKS][NT];
  {
    const int src = rows[32 * wid + l32];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = 16 * ks + 8 * h;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (src >= 0 && d0 < D) {
        const float* qp = qkv + (long long)src * ld + head * D + d0;
        a = *reinterpret_cast<const float4*>(qp);
        if (d0 + 4 < D) b = *reinterpret_cast<const float4*>(qp + 4);
      }
      // scale * log2(e) folded into q: the softmax exponentials are plain exp2
      const float qs = scale * 1.4426950408889634f;
      a.x *= qs; a.y *= qs; a.z *= qs; a.w *= qs;
      b.x *= qs; b.y *= qs; b.z *= qs; b.w *= qs;
      uint2 ta[NT], tb[NT];
      split(a, sq, ta);  // (|q * qs| <= |q|: the qkv bound holds)
      split(b, sq, tb);
#pragma unroll
      for (int q = 0; q < NT; ++q) qf[ks][q] = __builtin_bit_cast(bf16x8, (uintx4){ta[q].x, ta[q].y, tb[q].x, tb[q].y});
    }
  }
  for (int e = tid; e < KMAX * CH; e += 256) {
    const int row = e / CH, ch = e - row * CH;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int src = rows[row];
    if (src >= 0) v = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + C + head * D + 4 * ch);
    uint2 t[NT];
    split(v, sq, t);
    const int o = qk_off(row, ch >> 1) + ((ch & 1) << 3);
#pragma unroll
    for (int q = 0; q < NT; ++q) *reinterpret_cast<uint2*>(Ks + q * KMAX * QROW + o) = t[q];
  }
  for (int e = tid; e < (KMAX / 2) * CH; e += 256) {
    const int kp = e / CH, ch = e - kp * CH;
    const int row = 2 * kp;
    const int s0 = rows[row], s1 = rows[row + 1];
    float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
    if (s0 >= 0) v0 = *reinterpret_cast<const float4*>(qkv + (long long)s0 * ld + 2 * C + head * D + 4 * ch);
    if (s1 >= 0) v1 = *reinterpret_cast<const float4*>(qkv + (long long)s1 * ld + 2 * C + head * D + 4 * ch);
    uint2 t0[NT], t1[NT];
    split(v0, sq, t0);
    split(v1, sq, t1);
    const int kk = row & 15;  // even: keys row, row + 1 land on adjacent positions
    const int pos = (row & ~15) + 8 * ((kk >> 2) & 1) + (((kk >> 3) << 2) | (kk & 3));
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      unsigned* vt = reinterpret_cast<unsigned*>(Vt + (q * D + 4 * ch) * VST + (pos ^ (8 * vt_swz(4 * ch))));
      vt[0] = (t0[q].x & 0xffffu) | (t1[q].x << 16);
      vt[VST / 2] = (t0[q].x >> 16) | (t1[q].x & 0xffff0000u);
      vt[VST] = (t0[q].y & 0xffffu) | (t1[q].y << 16);
      vt[3 * VST / 2] = (t0[q].y >> 16) | (t1[q].y & 0xffff0000u);
    }
  }
  __syncthreads();

  // term products, smallest first
  constexpr int NP = F16 ? 3 : 6;
  constexpr int QA[6] = {F16 ? 1 : 2, F16 ? 0 : 1, 0, 1, 0, 0}, QB[6] = {0, 1, F16 ? 0 : 2, 0, 1, 0};
  constexpr int JS = ONE ? (F16 ? 2 : 3) : 0;  // first term product formed
  auto mfma = [](const bf16x8& a, const bf16x8& b, floatx16 c) -> floatx16 {
    if constexpr (F16) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  };
  // S^T[key][query] for this wave's 32 queries, 4 key blocks of 32
  floatx16 s[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      bf16x8 kf[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q)
        kf[q] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                               Ks + q * KMAX * QROW + qk_off(kb * 32 + l32, 2 * ks + h)));
#pragma unroll
      for (int j = JS; j < NP; ++j) s[kb] = mfma(kf[QA[j]], qf[ks][QB[j]], s[kb]);
    }
  }
  if constexpr (F16) {  // S was formed from sq-scaled q and k
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = s[kb][r] * iq * iq;
  }
  // softmax over keys (register axis + the other half-wave); keys >= Kwin only exist in short windows
  if (Kwin < KMAX) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (key >= Kwin) s[kb][r] = -INFINITY;
      }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = __builtin_amdgcn_exp2f(s[kb][r] - mx);
      s[kb][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float rinv = 1.f / sum;

  // O^T[dd][query] = sum_key V^T[dd][key] P^T[key][query]
  floatx16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      uint2 a[NT], b[NT];
      // unnormalised exp values (0, 1] (F16: scaled by 2^14); 1/sum is applied to O
      split(make_float4(s[kb][8 * st + 0], s[kb][8 * st + 1], s[kb][8 * st + 2], s[kb][8 * st + 3]), 16384.f, a);
      split(make_float4(s[kb][8 * st + 4], s[kb][8 * st + 5], s[kb][8 * st + 6], s[kb][8 * st + 7]), 16384.f, b);
      bf16x8 pf[NT], vf[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        pf[q] = __builtin_bit_cast(bf16x8, make_uint4(a[q].x, a[q].y, b[q].x, b[q].y));
        uint4 vv = make_uint4(0, 0, 0, 0);  // dd = l32 >= D: zero rows of V^T
        if (l32 < D) vv = *reinterpret_cast<const uint4*>(Vt + (q * D + l32) * VST + (((2 * (2 * kb + st) + h) ^ vt_swz(l32)) << 3));
        vf[q] = __builtin_bit_cast(bf16x8, vv);
      }
#pragma unroll
      for (int j = JS; j < NP; ++j) o = mfma(vf[QA[j]], pf[QB[j]], o);
    }

  const float oscale = F16 ? rinv * iq * (1.f / 16384.f) : rinv;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] *= oscale;
  // scatter: query 32*wid + l32 (lane column), dd rows (r&3) + 8(r>>2) + 4h
  const int qi = 32 * wid + l32;
  const int qpos = key_start + qi;
  if (qi < Kwin && qpos >= query_start) {
    float* dst = out + (long long)rows[qi] * C + head * D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dd = 8 * g + 4 * h;
      if (dd + 3 < D) {
        *reinterpret_cast<float4*>(dst + dd) = make_float4(o[4 * g + 0], o[4 * g + 1], o[4 * g + 2], o[4 * g + 3]);
      }
    }
  }
}


// window_attn_split_kernel<D, true> as a software pipeline over consecutive (window, head) items (window-major:
// all heads of a window back to back): a workgroup owns `ipw` consecutive items and, while it computes item i from
// LDS buffer i & 1, has item i + 1's row indices and q / k / v slices in flight into registers, split into the
// other buffer after item i's MFMAs -- the row gathers (the old kernel's whole latency: one item per workgroup,
// gather -> barrier -> compute -> store) overlap the compute.  Same arithmetic, same term order: outputs are bit
// for bit those of window_attn_split_kernel (test_window_attention_seq_bitwise).
template <int D>
__global__ void __launch_bounds__(256, 2)
window_attn_seq_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win,
                       int Kwin, int C, float scale, float* __restrict__ out,
                       const unsigned long long* __restrict__ qkv_amax, unsigned qkv_tag, int items, int ipw) {
  typedef _Float16 bf16x8 __attribute__((ext_vector_type(8)));
  constexpr int NT = 2;
  constexpr int KD = D == 16 ? 16 : 32;
  constexpr int NKS = KD / 16;
  constexpr int QROW = KD == 16 ? 48 : 64;
  constexpr int VST = 136;
  constexpr int QK_BYTES = NT * KMAX * QROW;
  constexpr int V_BYTES = NT * D * VST * 2;
  constexpr int BUF = QK_BYTES + V_BYTES;
  constexpr int CH = D / 4;
  constexpr int NK = (KMAX * CH + 255) / 256;         // K float4 per thread
  constexpr int NV = ((KMAX / 2) * CH + 255) / 256;   // V key pairs per thread
  float sq = 1.f, iq = 1.f;
  {
    const float m = sfx::read_amax(qkv_amax, qkv_tag);
    int e = 0;
    if (m > 0.f && m <= 3.4028235e38f) {
      (void)frexpf(m, &e);
      e = 15 - e;
      e = e > 126 ? 126 : (e < -126 ? -126 : e);
    }
    sq = ldexpf(1.f, e);
    iq = ldexpf(1.f, -e);
  }
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  auto qk_off = [](int r, int c) -> int {
    return KD == 16 ? r * 48 + c * 16 : r * 64 + (((c ^ (r >> 2)) & 3) << 4);
  };
  const int heads = C / D;
  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8);
  const int i0 = L * ipw, i1 = min(items, i0 + ipw);
  if (i0 >= i1) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;
  if (D < KD)  // K columns D..KD-1 of both buffers: zero once
    for (int rr = tid; rr < 2 * NT * KMAX; rr += 256) {
      const int b = rr / (NT * KMAX), r2 = rr - b * NT * KMAX;
      *reinterpret_cast<uint4*>(lds + b * BUF + qk_off(r2, D / 8)) = make_uint4(0, 0, 0, 0);
    }

  // ---- one item's gathered slices (registers) ----
  float4 kv[NK], vv0[NV], vv1[NV], qv[NKS][2];
  int qrow = -1;  // this lane's query point (output row) of the staged item
  auto fetch = [&](int it) {
    const int w = it / heads, head = it - w * heads;
    const int key_start = win[2 * w];
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int e = tid + 256 * j;
      const int row = e / CH, ch = e - row * CH;
      kv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < Kwin && e < KMAX * CH) {
        const int src = order[key_start + row];
        kv[j] = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + C + head * D + 4 * ch);
      }
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int e = tid + 256 * j;
      const int kp = e / CH, ch = e - kp * CH;
      vv0[j] = vv1[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < (KMAX / 2) * CH) {
        const int r0 = 2 * kp;
        if (r0 < Kwin)
          vv0[j] = *reinterpret_cast<const float4*>(qkv + (long long)order[key_start + r0] * ld + 2 * C + head * D + 4 * ch);
        if (r0 + 1 < Kwin)
          vv1[j] = *reinterpret_cast<const float4*>(qkv + (long long)order[key_start + r0 + 1] * ld + 2 * C + head * D +
                                                    4 * ch);
      }
    }
    const int qi = 32 * wid + l32;
    qrow = qi < Kwin ? order[key_start + qi] : -1;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = 16 * ks + 8 * h;
      qv[ks][0] = qv[ks][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (qrow >= 0 && d0 < D) {
        const float* qp = qkv + (long long)qrow * ld + head * D + d0;
        qv[ks][0] = *reinterpret_cast<const float4*>(qp);
        if (d0 + 4 < D) qv[ks][1] = *reinterpret_cast<const float4*>(qp + 4);
      }
    }
  };
  // ---- split into LDS buffer b (K, V^T) and the q fragments ----
  bf16x8 qf[NKS][NT];
  int qrow_s = -1;
  auto stage = [&](int b) {
    char* Ks = lds + b * BUF;
    unsigned short* Vt = reinterpret_cast<unsigned short*>(lds + b * BUF + QK_BYTES);
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int e = tid + 256 * j;
      if (e < KMAX * CH) {
        const int row = e / CH, ch = e - row * CH;
        uint2 t[NT];
        sfx::split2h(kv[j], sq, t);
        const int o = qk_off(row, ch >> 1) + ((ch & 1) << 3);
#pragma unroll
        for (int q = 0; q < NT; ++q) *reinterpret_cast<uint2*>(Ks + q * KMAX * QROW + o) = t[q];
      }
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int e = tid + 256 * j;
      if (e < (KMAX / 2) * CH) {
        const int kp = e / CH, ch = e - kp * CH;
        const int row = 2 * kp;
        uint2 t0[NT], t1[NT];
        sfx::split2h(vv0[j], sq, t0);
        sfx::split2h(vv1[j], sq, t1);
        const int kk = row & 15;
        const int pos = (row & ~15) + 8 * ((kk >> 2) & 1) + (((kk >> 3) << 2) | (kk & 3));
#pragma unroll
        for (int q = 0; q < NT; ++q) {
          unsigned* vt = reinterpret_cast<unsigned*>(Vt + (q * D + 4 * ch) * VST + (pos ^ (8 * vt_swz(4 * ch))));
          vt[0] = (t0[q].x & 0xffffu) | (t1[q].x << 16);
          vt[VST / 2] = (t0[q].x >> 16) | (t1[q].x & 0xffff0000u);
          vt[VST] = (t0[q].y & 0xffffu) | (t1[q].y << 16);
          vt[3 * VST / 2] = (t0[q].y >> 16) | (t1[q].y & 0xffff0000u);
        }
      }
    }
    const float qs = scale * 1.4426950408889634f;
    typedef unsigned uintx4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      float4 a = qv[ks][0], bb = qv[ks][1];
      a.x *= qs; a.y *= qs; a.z *= qs; a.w *= qs;
      bb.x *= qs; bb.y *= qs; bb.z *= qs; bb.w *= qs;
      uint2 ta[NT], tb[NT];
      sfx::split2h(a, sq, ta);
      sfx::split2h(bb, sq, tb);
#pragma unroll
      for (int q = 0; q < NT; ++q) qf[ks][q] = __builtin_bit_cast(bf16x8, (uintx4){ta[q].x, ta[q].y, tb[q].x, tb[q].y});
    }
    qrow_s = qrow;
  };

  fetch(i0);
  stage(0);
  __syncthreads();
  constexpr int QA[3] = {1, 0, 0}, QB[3] = {0, 1, 0};
  auto mfma = [](const bf16x8& a, const bf16x8& b, floatx16 c) -> floatx16 {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  };
#pragma unroll 1
  for (int it = i0; it < i1; ++it) {
    const int b = (it - i0) & 1;
    const int w = it / heads, head = it - w * heads;
    const int key_start = win[2 * w], query_start = win[2 * w + 1];
    if (it + 1 < i1) fetch(it + 1);  // next item's slices in flight during this item's compute
    const char* Ks = lds + b * BUF;
    const unsigned short* Vt = reinterpret_cast<const unsigned short*>(lds + b * BUF + QK_BYTES);
    floatx16 sacc[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kb][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        bf16x8 kf[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q)
          kf[q] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                 Ks + q * KMAX * QROW + qk_off(kb * 32 + l32, 2 * ks + h)));
#pragma unroll
        for (int j = 0; j < 3; ++j) sacc[kb] = mfma(kf[QA[j]], qf[ks][QB[j]], sacc[kb]);
      }
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kb][r] = sacc[kb][r] * iq * iq;
    if (Kwin < KMAX) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (key >= Kwin) sacc[kb][r] = -INFINITY;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[kb][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(sacc[kb][r] - mx);
        sacc[kb][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 32, 64);
    const float rinv = 1.f / sum;
    floatx16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        uint2 a[NT], bb[NT];
        sfx::split2h(make_float4(sacc[kb][8 * st + 0], sacc[kb][8 * st + 1], sacc[kb][8 * st + 2], sacc[kb][8 * st + 3]),
                     16384.f, a);
        sfx::split2h(make_float4(sacc[kb][8 * st + 4], sacc[kb][8 * st + 5], sacc[kb][8 * st + 6], sacc[kb][8 * st + 7]),
                     16384.f, bb);
        bf16x8 pf[NT], vf[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) {
          pf[q] = __builtin_bit_cast(bf16x8, make_uint4(a[q].x, a[q].y, bb[q].x, bb[q].y));
          uint4 v4 = make_uint4(0, 0, 0, 0);
          if (l32 < D) v4 = *reinterpret_cast<const uint4*>(Vt + (q * D + l32) * VST + (((2 * (2 * kb + st) + h) ^ vt_swz(l32)) << 3));
          vf[q] = __builtin_bit_cast(bf16x8, v4);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) o = mfma(vf[QA[j]], pf[QB[j]], o);
      }
    const float oscale = rinv * iq * (1.f / 16384.f);
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] *= oscale;
    const int qi = 32 * wid + l32;
    const int qpos = key_start + qi;
    if (qi < Kwin && qpos >= query_start) {
      float* dst = out + (long long)qrow_s * C + head * D;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 8 * g + 4 * h;
        if (dd + 3 < D) *reinterpret_cast<float4*>(dst + dd) = make_float4(o[4 * g + 0], o[4 * g + 1], o[4 * g + 2], o[4 * g + 3]);
      }
    }
    if (it + 1 < i1) stage(b ^ 1);
    __syncthreads();
  }
}


// Flash mode on split MFMA terms (default for sfx_window_attention_varlen): window_attn_split_kernel's
// dataflow (per-lane query fragments, K / V^T term images, S^T = K Q^T and O^T = V^T P^T on fp16x2 or bf16x3
// terms) with the window's keys streamed in 128-key blocks and an online softmax: the running maximum
// rescales the accumulator by exp2(m_old - m_new), so every block's probabilities stay in (0, 1] (the 2^14
// fp16 scale of P holds).  One workgroup per (window, 128-query block, head), XCD-aware numbering.
template <int D, bool F16>
__global__ void __launch_bounds__(256, D == 16 ? 4 : 3)
window_attn_split_flash_kernel(const float* __restrict__ qkv, const int* __restrict__ order,
                               const int* __restrict__ win3, int qblocks, int C, float scale, float* __restrict__ out,
                               const unsigned long long* __restrict__ qkv_amax, unsigned qkv_tag, int nwin) {
  typedef typename std::conditional<F16, _Float16, __bf16>::type elem_t;
  typedef elem_t bf16x8 __attribute__((ext_vector_type(8)));  // (fragment type: bf16 or fp16 terms)
  constexpr int NT = F16 ? 2 : 3;            // terms per operand
  constexpr int KD = D == 16 ? 16 : 32;
  constexpr int NKS = KD / 16;
  constexpr int QROW = KD == 16 ? 48 : 64;  // bytes per Q/K term row
  constexpr int VST = 136;                  // V^T row stride (16-bit elements)
  constexpr int QK_BYTES = NT * KMAX * QROW;
  constexpr int V_BYTES = NT * D * VST * 2;
  // operand scales (F16): qkv by sq, probabilities by 2^14
  float sq = 1.f, iq = 1.f;
  if constexpr (F16) {
    const float m = sfx::read_amax(qkv_amax, qkv_tag);
    int e = 0;
    if (m > 0.f && m <= 3.4028235e38f) {
      (void)frexpf(m, &e);
      e = 15 - e;
      e = e > 126 ? 126 : (e < -126 ? -126 : e);
    }
    sq = ldexpf(1.f, e);
    iq = ldexpf(1.f, -e);
  }
  auto split = [&](float4 v, float sc, uint2 (&t)[NT]) {
    if constexpr (F16) sfx::split2h(v, sc, t); else sfx::split3(v, t);
  };
  __shared__ __attribute__((aligned(16))) char lds[QK_BYTES + V_BYTES];
  __shared__ int rows[KMAX];   // keys of the current block
  __shared__ int qrows[KMAX];  // this workgroup's queries
  char* Ks = lds;
  unsigned short* Vt = reinterpret_cast<unsigned short*>(lds + QK_BYTES);
  // byte offset of 16-byte chunk c of term row r
  auto qk_off = [](int r, int c) -> int {
    return KD == 16 ? r * 48 + c * 16 : r * 64 + (((c ^ (r >> 2)) & 3) << 4);
  };

  // XCD-aware numbering over a 1-D grid padded to a multiple of 8: consecutive blocks go round-robin to the 8
  // XCDs, so logical id L = xcd * (grid / 8) + slot puts all heads of a window on one XCD back to back -- the
  // 128-byte qkv lines its heads share (d = 16: two heads per line) are fetched from HBM once into that L2.
  const int heads = C / D;
  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8);
  if (L >= nwin * qblocks * heads) return;
  const int wq = L / heads, head = L - wq * heads;
  const int w = wq / qblocks, qb = wq - w * qblocks;
  const int key_start = win3[3 * w], query_start = win3[3 * w + 1], count = win3[3 * w + 2];
  const int q0 = qb * KMAX;
  if (q0 >= count || key_start + q0 + KMAX <= query_start) return;  // workgroup-uniform, before any barrier
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  if (tid < KMAX) qrows[tid] = q0 + tid < count ? order[key_start + q0 + tid] : -1;
  // zero padding: K columns D..KD-1 (never written by the staging below)
  if (D < KD)
    for (int rr = tid; rr < NT * KMAX; rr += 256)  // term rows, term-major
      *reinterpret_cast<uint4*>(Ks + qk_off(rr, D / 8)) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  // gather + split, one matrix at a time (wave-uniform paths): q, k rows as KMAX x D/4 float4; v as
  // key pairs x D/4 float4 so the transposed V^T writes are whole dwords (keys 2m, 2m+1 are adjacent
  // in the permuted order)
  constexpr int CH = D / 4;
  typedef unsigned uintx4 __attribute__((ext_vector_type(4)));
  // this lane's query slices (B operand of S^T = K Q^T): dd = 16 ks + 8h + j, zero past D
  bf16x8 qf[NKS][NT];
  {
    const int src = qrows[32 * wid + l32];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = 16 * ks + 8 * h;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (src >= 0 && d0 < D) {
        const float* qp = qkv + (long long)src * ld + head * D + d0;
        a = *reinterpret_cast<const float4*>(qp);
        if (d0 + 4 < D) b = *reinterpret_cast<const float4*>(qp + 4);
      }
      // scale * log2(e) folded into q: the softmax exponentials are plain exp2
      const float qs = scale * 1.4426950408889634f;
      a.x *= qs; a.y *= qs; a.z *= qs; a.w *= qs;
      b.x *= qs; b.y *= qs; b.z *= qs; b.w *= qs;
      uint2 ta[NT], tb[NT];
      split(a, sq, ta);  // (|q * qs| <= |q|: the qkv bound holds)
      split(b, sq, tb);
#pragma unroll
      for (int q = 0; q < NT; ++q) qf[ks][q] = __builtin_bit_cast(bf16x8, (uintx4){ta[q].x, ta[q].y, tb[q].x, tb[q].y});
    }
  }
  // term products, smallest first
  constexpr int NP = F16 ? 3 : 6;
  constexpr int QA[6] = {F16 ? 1 : 2, F16 ? 0 : 1, 0, 1, 0, 0}, QB[6] = {0, 1, F16 ? 0 : 2, 0, 1, 0};
  auto mfma = [](const bf16x8& a, const bf16x8& b, floatx16 c) -> floatx16 {
    if constexpr (F16) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  };
  float m_run = -INFINITY, l_run = 0.f;
  floatx16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;

  for (int k0 = 0; k0 < count; k0 += KMAX) {
    const int nk = min(KMAX, count - k0);
    __syncthreads();  // the previous block's fragment reads are done
    if (tid < KMAX) rows[tid] = tid < nk ? order[key_start + k0 + tid] : -1;
    __syncthreads();
    for (int e = tid; e < KMAX * CH; e += 256) {
      const int row = e / CH, ch = e - row * CH;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int src = rows[row];
      if (src >= 0) v = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + C + head * D + 4 * ch);
      uint2 t[NT];
      split(v, sq, t);
      const int o = qk_off(row, ch >> 1) + ((ch & 1) << 3);
#pragma unroll
      for (int q = 0; q < NT; ++q) *reinterpret_cast<uint2*>(Ks + q * KMAX * QROW + o) = t[q];
    }
    for (int e = tid; e < (KMAX / 2) * CH; e += 256) {
      const int kp = e / CH, ch = e - kp * CH;
      const int row = 2 * kp;
      const int s0 = rows[row], s1 = rows[row + 1];
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (s0 >= 0) v0 = *reinterpret_cast<const float4*>(qkv + (long long)s0 * ld + 2 * C + head * D + 4 * ch);
      if (s1 >= 0) v1 = *reinterpret_cast<const float4*>(qkv + (long long)s1 * ld + 2 * C + head * D + 4 * ch);
      uint2 t0[NT], t1[NT];
      split(v0, sq, t0);
      split(v1, sq, t1);
      const int kk = row & 15;  // even: keys row, row + 1 land on adjacent positions
      const int pos = (row & ~15) + 8 * ((kk >> 2) & 1) + (((kk >> 3) << 2) | (kk & 3));
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        unsigned* vt = reinterpret_cast<unsigned*>(Vt + (q * D + 4 * ch) * VST + (pos ^ (8 * vt_swz(4 * ch))));
        vt[0] = (t0[q].x & 0xffffu) | (t1[q].x << 16);
        vt[VST / 2] = (t0[q].x >> 16) | (t1[q].x & 0xffff0000u);
        vt[VST] = (t0[q].y & 0xffffu) | (t1[q].y << 16);
        vt[3 * VST / 2] = (t0[q].y >> 16) | (t1[q].y & 0xffff0000u);
      }
    }
    __syncthreads();

    // S^T[key][query] for this wave's 32 queries, 4 key blocks of 32
    floatx16 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        bf16x8 kf[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q)
          kf[q] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                 Ks + q * KMAX * QROW + qk_off(kb * 32 + l32, 2 * ks + h)));
#pragma unroll
        for (int j = 0; j < NP; ++j) s[kb] = mfma(kf[QA[j]], qf[ks][QB[j]], s[kb]);
      }
    }
    if constexpr (F16) {  // S was formed from sq-scaled q and k
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kb][r] = s[kb][r] * iq * iq;
    }
    // online softmax over this key block (register axis + the other half-wave); keys >= nk are padding
    if (nk < KMAX) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (key >= nk) s[kb][r] = -INFINITY;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    mx = fmaxf(mx, m_run);  // finite: every block holds at least one key
    const float corr = __builtin_amdgcn_exp2f(m_run - mx);
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[kb][r] - mx);
        s[kb][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 32, 64);
    l_run = l_run * corr + sum;
    m_run = mx;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] *= corr;

    // O^T[dd][query] += sum_key V^T[dd][key] P^T[key][query]
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        uint2 a[NT], b[NT];
        // unnormalised exp values (0, 1] (F16: scaled by 2^14); 1/sum is applied to O
        split(make_float4(s[kb][8 * st + 0], s[kb][8 * st + 1], s[kb][8 * st + 2], s[kb][8 * st + 3]), 16384.f, a);
        split(make_float4(s[kb][8 * st + 4], s[kb][8 * st + 5], s[kb][8 * st + 6], s[kb][8 * st + 7]), 16384.f, b);
        bf16x8 pf[NT], vf[NT];
#pragma unroll
        for (int q = 0; q < NT; ++q) {
          pf[q] = __builtin_bit_cast(bf16x8, make_uint4(a[q].x, a[q].y, b[q].x, b[q].y));
          uint4 vv = make_uint4(0, 0, 0, 0);  // dd = l32 >= D: zero rows of V^T
          if (l32 < D) vv = *reinterpret_cast<const uint4*>(Vt + (q * D + l32) * VST + (((2 * (2 * kb + st) + h) ^ vt_swz(l32)) << 3));
          vf[q] = __builtin_bit_cast(bf16x8, vv);
        }
#pragma unroll
        for (int j = 0; j < NP; ++j) o = mfma(vf[QA[j]], pf[QB[j]], o);
      }
  }  // key blocks

  const float rinv = 1.f / l_run;
  const float oscale = F16 ? rinv * iq * (1.f / 16384.f) : rinv;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] *= oscale;
  // scatter: query 32*wid + l32 (lane column), dd rows (r&3) + 8(r>>2) + 4h
  const int qi = q0 + 32 * wid + l32;
  if (qi < count && key_start + qi >= query_start) {
    float* dst = out + (long long)qrows[32 * wid + l32] * C + head * D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dd = 8 * g + 4 * h;
      if (dd + 3 < D) {
        *reinterpret_cast<float4*>(dst + dd) = make_float4(o[4 * g + 0], o[4 * g + 1], o[4 * g + 2], o[4 * g + 3]);
      }
    }
  }
}


// ---- backward (training, configs C/D) ---------------------------------------------------------------
// Autograd of the non-flash attention math of visualize.py:140-179 for one (window, head):
//   dV = P^T dO ; dP = dO V^T ; dS = P * (dP - rowsum(dO * O)) ; dQ = scale * dS K ; dK = dS^T (scale*Q)
// Phase A (query on the lane column, S^T = K Q^T as in the forward): softmax statistics, O, Delta, dS^T
// and dQ -- every query row belongs to exactly one window, so dQ is a plain store.  Phase B (key on the
// lane column, S = Q K^T recomputed): dV and dK summed over the window's queries; a key can sit in two
// windows (the ragged last window re-uses the K - n%K points before it), so they are accumulated with
// float atomics into dqkv, which the caller zero-fills.  Padding queries (positions < query_start of the
// last window) carry dO = 0 and contribute nothing, exactly as their discarded outputs in the reference.
template <int D>
__global__ void __launch_bounds__(256, 2)
window_attn_bwd_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win,
                       int Kwin, int C, float scale, const float* __restrict__ dout, float* __restrict__ dqkv) {
  // One row stride for all four operands: 36 floats = 32 (+4) columns, zero beyond D.  ds_read_b128 row
  // reads (S, dP) are conflict-free at stride 36 and the MFMA A-operand column reads (V^T, K^T, dO^T, Q^T
  // with dd = lane) need no masking for dd >= D.  4 x 18 KB LDS -> 2 workgroups per CU.
  constexpr int DP = 36;
  constexpr int HALF = D / 2;
  __shared__ __attribute__((aligned(16))) float Qs[KMAX * DP];
  __shared__ __attribute__((aligned(16))) float Ks[KMAX * DP];
  __shared__ __attribute__((aligned(16))) float Vs[KMAX * DP];
  __shared__ __attribute__((aligned(16))) float dOs[KMAX * DP];
  __shared__ float st_max[KMAX], st_rinv[KMAX], st_delta[KMAX];
  __shared__ int rows[KMAX];

  const int w = blockIdx.x, head = blockIdx.y;
  const int key_start = win[2 * w], query_start = win[2 * w + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  if (tid < KMAX) rows[tid] = tid < Kwin ? order[key_start + tid] : -1;
  __syncthreads();
  // gather q/k/v/dO rows of this head (zero rows past Kwin, zero dO for padding queries, zero columns >= D)
  constexpr int CH = 8;  // float4 per padded row (32 columns)
  for (int e = tid; e < KMAX * 4 * CH; e += 256) {
    const int row = e / (4 * CH);
    const int rem = e - row * 4 * CH;
    const int mat = rem / CH, ch = rem - mat * CH;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int src = rows[row];
    if (4 * ch < D && src >= 0) {
      if (mat < 3)
        v = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + mat * C + head * D + 4 * ch);
      else if (key_start + row >= query_start)
        v = *reinterpret_cast<const float4*>(dout + (long long)src * C + head * D + 4 * ch);
    }
    float* dst = mat == 0 ? Qs : mat == 1 ? Ks : mat == 2 ? Vs : dOs;
    if (mat == 0) {
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
    }
    *reinterpret_cast<float4*>(&dst[row * DP + 4 * ch]) = v;
  }
  __syncthreads();

  // ---------------- phase A: this wave's 32 queries on the lane columns ----------------
  const int qi = 32 * wid + l32;
  floatx16 s[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
  {
    const float* qrow = &Qs[qi * DP + h * HALF];
#pragma unroll
    for (int c = 0; c < HALF / 4; ++c) {
      const float4 qv = *reinterpret_cast<const float4*>(qrow + 4 * c);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float4 kv = *reinterpret_cast<const float4*>(&Ks[(kb * 32 + l32) * DP + h * HALF + 4 * c]);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qv.x, s[kb], 0, 0, 0);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qv.y, s[kb], 0, 0, 0);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qv.z, s[kb], 0, 0, 0);
        s[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qv.w, s[kb], 0, 0, 0);
      }
    }
  }
  if (Kwin < KMAX) {
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (key >= Kwin) s[kb][r] = -INFINITY;
      }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kb][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = __expf(s[kb][r] - mx);
      s[kb][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float rinv = 1.f / sum;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] *= rinv;  // P^T (same normalisation as the forward)
  // O^T[dd][q] (forward recompute) -> Delta_q = sum_dd O[q][dd] dO[q][dd]
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const float* vcol = &Vs[4 * h * DP + l32];
  const float* kcol = &Ks[4 * h * DP + l32];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int st = 0; st < 16; ++st)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vcol[(kb * 32 + (st & 3) + 8 * (st >> 2)) * DP], s[kb][st], acc, 0, 0,
                                                 0);
  float delta = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) delta += acc[r] * dOs[qi * DP + (r & 3) + 8 * (r >> 2) + 4 * h];
  delta += __shfl_xor(delta, 32, 64);
  // per key block: dP^T = V dO^T, dS^T = P^T (dP^T - Delta), dQ^T += K^T dS^T
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;  // now dQ^T
  const float* grow = &dOs[qi * DP + h * HALF];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    floatx16 dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = 0.f;
#pragma unroll
    for (int c = 0; c < HALF / 4; ++c) {
      const float4 gv = *reinterpret_cast<const float4*>(grow + 4 * c);
      const float4 vv = *reinterpret_cast<const float4*>(&Vs[(kb * 32 + l32) * DP + h * HALF + 4 * c]);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.x, gv.x, dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.y, gv.y, dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.z, gv.z, dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.w, gv.w, dp, 0, 0, 0);
    }
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const float ds = s[kb][st] * (dp[st] - delta);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kcol[(kb * 32 + (st & 3) + 8 * (st >> 2)) * DP], ds, acc, 0, 0, 0);
    }
  }
  const int qpos = key_start + qi;
  if (qi < Kwin && qpos >= query_start) {
    float* dst = dqkv + (long long)rows[qi] * ld + head * D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dd = 8 * g + 4 * h;
      if (dd + 3 < D)
        *reinterpret_cast<float4*>(dst + dd) =
            make_float4(acc[4 * g + 0] * scale, acc[4 * g + 1] * scale, acc[4 * g + 2] * scale, acc[4 * g + 3] * scale);
    }
  }
  if (h == 0) {
    st_max[qi] = mx;
    st_rinv[qi] = rinv;
    st_delta[qi] = delta;
  }
  __syncthreads();

  // ---------------- phase B: this wave's 32 keys on the lane columns ----------------
  const int kk = 32 * wid + l32;
  floatx16 dk, dv;
#pragma unroll
  for (int r = 0; r < 16; ++r) dk[r] = dv[r] = 0.f;
  const bool key_ok = kk < Kwin;
  const float* krow = &Ks[kk * DP + h * HALF];
  const float* vrow = &Vs[kk * DP + h * HALF];
  const float* gcol = &dOs[4 * h * DP + l32];
  const float* qcol = &Qs[4 * h * DP + l32];
#pragma unroll 1
  for (int qb = 0; qb < 4; ++qb) {
    floatx16 sb, pb;
#pragma unroll
    for (int r = 0; r < 16; ++r) sb[r] = pb[r] = 0.f;
    const float* qrow = &Qs[(qb * 32 + l32) * DP + h * HALF];
    const float* grw = &dOs[(qb * 32 + l32) * DP + h * HALF];
#pragma unroll
    for (int c = 0; c < HALF / 4; ++c) {
      const float4 qv = *reinterpret_cast<const float4*>(qrow + 4 * c);
      const float4 gv = *reinterpret_cast<const float4*>(grw + 4 * c);
      const float4 kv = *reinterpret_cast<const float4*>(krow + 4 * c);
      const float4 vv = *reinterpret_cast<const float4*>(vrow + 4 * c);
      sb = __builtin_amdgcn_mfma_f32_32x32x2f32(qv.x, kv.x, sb, 0, 0, 0);
      sb = __builtin_amdgcn_mfma_f32_32x32x2f32(qv.y, kv.y, sb, 0, 0, 0);
      sb = __builtin_amdgcn_mfma_f32_32x32x2f32(qv.z, kv.z, sb, 0, 0, 0);
      sb = __builtin_amdgcn_mfma_f32_32x32x2f32(qv.w, kv.w, sb, 0, 0, 0);
      pb = __builtin_amdgcn_mfma_f32_32x32x2f32(gv.x, vv.x, pb, 0, 0, 0);
      pb = __builtin_amdgcn_mfma_f32_32x32x2f32(gv.y, vv.y, pb, 0, 0, 0);
      pb = __builtin_amdgcn_mfma_f32_32x32x2f32(gv.z, vv.z, pb, 0, 0, 0);
      pb = __builtin_amdgcn_mfma_f32_32x32x2f32(gv.w, vv.w, pb, 0, 0, 0);
    }
    // sb[r] = S[q][kk], pb[r] = dP[q][kk] for q = qb*32 + (r&3) + 8(r>>2) + 4h
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int q = qb * 32 + (st & 3) + 8 * (st >> 2) + 4 * h;
      const float P = key_ok ? __expf(sb[st] - st_max[q]) * st_rinv[q] : 0.f;
      const float dS = P * (pb[st] - st_delta[q]);
      const int qo = (qb * 32 + (st & 3) + 8 * (st >> 2)) * DP;  // + 4h folded into gcol / qcol
      dv = __builtin_amdgcn_mfma_f32_32x32x2f32(gcol[qo], P, dv, 0, 0, 0);
      dk = __builtin_amdgcn_mfma_f32_32x32x2f32(qcol[qo], dS, dk, 0, 0, 0);
    }
  }
  // dK / dV leave through LDS so that each store instruction writes whole row segments (a lane-per-key
  // layout would touch 64 rows per instruction).  Keys in the overlap of the ragged last window with its
  // predecessor receive contributions from both windows and are added atomically; every other key is owned
  // by this window alone and stored plainly.
  __syncthreads();  // all waves done reading Q/K/V/dO
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int dd = (r & 3) + 8 * (r >> 2) + 4 * h;
    Qs[kk * DP + dd] = dk[r];
    Vs[kk * DP + dd] = dv[r];
  }
  __syncthreads();
  const int next_ks = (w + 1 < (int)gridDim.x) ? win[2 * (w + 1)] : 0x7fffffff;
  constexpr int DC = D / 4;
  for (int e = tid; e < Kwin * 2 * DC; e += 256) {
    const int row = e / (2 * DC);
    const int rem = e - row * 2 * DC;
    const int mat = rem / DC, ch = rem - mat * DC;
    const float4 v = *reinterpret_cast<const float4*>(&(mat == 0 ? Qs : Vs)[row * DP + 4 * ch]);
    float* dst = dqkv + (long long)rows[row] * ld + (mat + 1) * C + head * D + 4 * ch;
    const int pos = key_start + row;
    if (pos < query_start || pos >= next_ks) {
      atomicAdd(dst + 0, v.x);
      atomicAdd(dst + 1, v.y);
      atomicAdd(dst + 2, v.z);
      atomicAdd(dst + 3, v.w);
    } else {
      *reinterpret_cast<float4*>(dst) = v;
    }
  }
}

// ---- fp16x2 backward (default) -----------------------------------------------------------------------------
// The same autograd as window_attn_bwd_kernel in two passes over the (window, head) items, on
// v_mfma_f32_32x32x16_f16 with every operand as two fp16 terms (sfx::split2h) of a power-of-two-scaled value and
// three term products per block (the forward's F16 scheme):
//   query pass (lanes = this wave's 32 queries):  S^T = K Q^T -> softmax max and 1/sum ; Delta_q = dO_q . O_q from
//     the forward output (= rowsum(P o dP)) ; per 32-key block dP^T = V dO^T, dS^T = P^T (dP^T - Delta) and
//     dQ^T += K^T dS^T with dS^T straight from registers as the B operand (as P^T in the forward) ; dQ stored plainly
//     (each query belongs to one window) and (max, 1/sum, Delta) written per (query, head) for the key pass;
//   key pass (lanes = this wave's 32 keys): per 32-query block S = Q K^T and dP = dO V^T recomputed, P from the
//     stored statistics, dS = P (dP - Delta) ; dV^T += dO^T P and dK^T += Q^T dS from registers.
// Scales: q, k, v and dO of an item by powers of two putting the item's largest magnitude in [2^14, 2^15); P (<= 1)
// by 2^14; dS by one power of two per (lane column, 32-row block), its block product unscaled before it joins the
// accumulator.  Every MFMA is a 16-deep step of 3 products, against 8 steps of v_mfma_f32_32x32x2_f32 per 16 in the
// exact kernel; recomputing S and dP in the key pass is what keeps both passes' contractions on the register axis.
// LDS per item: row images [2 terms][128][KD] (as the forward's K image) and transposed images [2][D][136] with the
// keys (queries) of each 16-group in the B-operand register order (as the forward's V^T).
template <int KD>
__device__ __forceinline__ int bwd_row_off(int r, int c) {  // byte offset of 16-byte chunk c of term row r
  return KD == 16 ? r * 48 + c * 16 : r * 64 + (((c ^ (r >> 2)) & 3) << 4);
}
// power of two s with m * s in [2^14, 2^15) (1 for m == 0 or non-finite m); inv = 1 / s
__device__ __forceinline__ float bwd_pow2(float m, float& inv) {
  int e = 0;
  if (m > 0.f && m <= 3.4028235e38f) {
    (void)frexpf(m, &e);
    e = 15 - e;
    e = e > 126 ? 126 : (e < -126 ? -126 : e);
  }
  inv = ldexpf(1.f, -e);
  return ldexpf(1.f, e);
}
__device__ __forceinline__ float amax4(float4 v) {
  return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}
// workgroup-wide max of 4 values (256 threads, one barrier)
__device__ __forceinline__ float4 bwd_wg_max4(float4 m, float4* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    m.x = fmaxf(m.x, __shfl_xor(m.x, o, 64));
    m.y = fmaxf(m.y, __shfl_xor(m.y, o, 64));
    m.z = fmaxf(m.z, __shfl_xor(m.z, o, 64));
    m.w = fmaxf(m.w, __shfl_xor(m.w, o, 64));
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float4 r = red[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    const float4 t = red[i];
    r = make_float4(fmaxf(r.x, t.x), fmaxf(r.y, t.y), fmaxf(r.z, t.z), fmaxf(r.w, t.w));
  }
  return r;
}
// two fp16 terms of 8 scaled values -> B-operand fragments
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void bwd_frag(float4 a, float4 b, float s, f16x8 (&f)[2]) {
  uint2 ta[2], tb[2];
  sfx::split2h(a, s, ta);
  sfx::split2h(b, s, tb);
#pragma unroll
  for (int t = 0; t < 2; ++t) f[t] = __builtin_bit_cast(f16x8, make_uint4(ta[t].x, ta[t].y, tb[t].x, tb[t].y));
}
// ONE (sfx_set_precision(1), the reference's autocast class): the leading product only
template <bool ONE = false>
__device__ __forceinline__ floatx16 mfma3(const f16x8 (&a)[2], const f16x8 (&b)[2], floatx16 c) {
  if constexpr (ONE) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], c, 0, 0, 0);  // smallest first
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
}
// a lane's 8 (or fewer, zero-padded past D) values of row `src`, columns d0 .. d0 + 7
template <int D>
__device__ __forceinline__ void bwd_load8(const float* p, int d0, bool ok, float4& a, float4& b) {
  a = make_float4(0.f, 0.f, 0.f, 0.f);
  b = a;
  if (ok && d0 < D) {
    a = *reinterpret_cast<const float4*>(p + d0);
    if (d0 + 4 < D) b = *reinterpret_cast<const float4*>(p + d0 + 4);
  }
}
// row image + transposed image of a pair of rows (2p, 2p + 1), float4 column chunk ch, terms of x * s
template <int D, int KD>
__device__ __forceinline__ void bwd_stage_pair(char* rimg, unsigned short* timg, int row, int ch, float4 v0, float4 v1,
                                               float s) {
  constexpr int QROW = KD == 16 ? 48 : 64, VST = 136;
  uint2 t0[2], t1[2];
  sfx::split2h(v0, s, t0);
  sfx::split2h(v1, s, t1);
  const int o0 = bwd_row_off<KD>(row, ch >> 1) + ((ch & 1) << 3);
  const int o1 = bwd_row_off<KD>(row + 1, ch >> 1) + ((ch & 1) << 3);
  const int kk = row & 15;  // even: rows row, row + 1 land on adjacent positions
  const int pos = (row & ~15) + 8 * ((kk >> 2) & 1) + (((kk >> 3) << 2) | (kk & 3));
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    *reinterpret_cast<uint2*>(rimg + q * KMAX * QROW + o0) = t0[q];
    *reinterpret_cast<uint2*>(rimg + q * KMAX * QROW + o1) = t1[q];
    unsigned* vt = reinterpret_cast<unsigned*>(timg + (q * D + 4 * ch) * VST + (pos ^ (8 * vt_swz(4 * ch))));
    vt[0] = (t0[q].x & 0xffffu) | (t1[q].x << 16);
    vt[VST / 2] = (t0[q].x >> 16) | (t1[q].x & 0xffff0000u);
    vt[VST] = (t0[q].y & 0xffffu) | (t1[q].y << 16);
    vt[3 * VST / 2] = (t0[q].y >> 16) | (t1[q].y & 0xffff0000u);
  }
}
template <int KD>
__device__ __forceinline__ void bwd_stage_row(char* rimg, int row, int ch, float4 v, float s) {
  constexpr int QROW = KD == 16 ? 48 : 64;
  uint2 t[2];
  sfx::split2h(v, s, t);
  const int o = bwd_row_off<KD>(row, ch >> 1) + ((ch & 1) << 3);
#pragma unroll
  for (int q = 0; q < 2; ++q) *reinterpret_cast<uint2*>(rimg + q * KMAX * QROW + o) = t[q];
}
template <int KD>
__device__ __forceinline__ void bwd_row_frag(const char* rimg, int row, int c, f16x8 (&f)[2]) {
  constexpr int QROW = KD == 16 ? 48 : 64;
#pragma unroll
  for (int q = 0; q < 2; ++q)
    f[q] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(rimg + q * KMAX * QROW + bwd_row_off<KD>(row, c)));
}
// A fragment of a transposed image: lane row dd = l32 (zero past D), 8 keys of 16-step `step` from half h
template <int D>
__device__ __forceinline__ void bwd_tr_frag(const unsigned short* timg, int l32, int step, int h, f16x8 (&f)[2]) {
  constexpr int VST = 136;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (l32 < D) v = *reinterpret_cast<const uint4*>(timg + (q * D + l32) * VST + (((2 * step + h) ^ vt_swz(l32)) << 3));
    f[q] = __builtin_bit_cast(f16x8, v);
  }
}

template <int D, bool ONE = false>
__global__ void __launch_bounds__(256, 3)
window_attn_bwd_q_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win,
                         int Kwin, int C, float scale, const float* __restrict__ attn_out,
                         const float* __restrict__ dout, float* __restrict__ dqkv, float4* __restrict__ stats,
                         int nwin) {
  constexpr int KD = D == 16 ? 16 : 32, NKS = KD / 16, QROW = KD == 16 ? 48 : 64, VST = 136;
  constexpr int RB = 2 * KMAX * QROW, TB = 2 * D * VST * 2;
  constexpr int CH = D / 4, NE = (KMAX / 2) * CH, NIT = (NE + 255) / 256;
  __shared__ __attribute__((aligned(16))) char lds[2 * RB + TB];
  __shared__ int rows[KMAX];
  __shared__ float4 red[4];
  char* Kr = lds;
  char* Vr = lds + RB;
  unsigned short* Kt = reinterpret_cast<unsigned short*>(lds + 2 * RB);

  const int heads = C / D;
  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8);  // XCD-aware, as the forward
  if (L >= nwin * heads) return;
  const int w = L / heads, head = L - w * heads;
  const int key_start = win[2 * w], query_start = win[2 * w + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  if (tid < KMAX) rows[tid] = tid < Kwin ? order[key_start + tid] : -1;
  if (D < KD)  // zero K / V columns D..KD-1
    for (int rr = tid; rr < 4 * KMAX; rr += 256)
      *reinterpret_cast<uint4*>(lds + (rr >> 8) * RB + ((rr >> 7) & 1) * KMAX * QROW + bwd_row_off<KD>(rr & 127, D / 8)) =
          make_uint4(0, 0, 0, 0);
  __syncthreads();
  // dqkv is not zero-filled by the caller: the key pass stores every key's dK / dV plainly except the keys a ragged
  // last window shares with its predecessor (positions key_start .. query_start - 1), which both windows add
  // atomically -- this window zeroes this head's slice of them here, a launch ahead of every key-pass add
  for (int e = tid; e < (query_start - key_start) * 2 * (D / 4); e += 256) {
    const int row = e / (2 * (D / 4)), rem = e - row * 2 * (D / 4);
    const int mat = rem / (D / 4), ch = rem - mat * (D / 4);
    *reinterpret_cast<float4*>(dqkv + (long long)rows[row] * ld + (mat + 1) * C + head * D + 4 * ch) =
        make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // this lane's query: q and dO slices dd = 16 ks + 8h .. +7 (B operands of S^T and dP^T) and Delta = dO . O
  const int qi = 32 * wid + l32;
  const int qsrc = rows[qi];
  const bool qown = qsrc >= 0 && key_start + qi >= query_start;
  float4 qa[NKS][2], ga[NKS][2];
  float delta = 0.f;
  float4 mx4 = make_float4(0.f, 0.f, 0.f, 0.f);  // (q, k, v, dO)
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int d0 = 16 * ks + 8 * h;
    bwd_load8<D>(qkv + (long long)(qsrc < 0 ? 0 : qsrc) * ld + head * D, d0, qsrc >= 0, qa[ks][0], qa[ks][1]);
    bwd_load8<D>(dout + (long long)(qsrc < 0 ? 0 : qsrc) * C + head * D, d0, qown, ga[ks][0], ga[ks][1]);
    float4 oa, ob;
    bwd_load8<D>(attn_out + (long long)(qsrc < 0 ? 0 : qsrc) * C + head * D, d0, qown, oa, ob);
    delta += ga[ks][0].x * oa.x + ga[ks][0].y * oa.y + ga[ks][0].z * oa.z + ga[ks][0].w * oa.w +
             ga[ks][1].x * ob.x + ga[ks][1].y * ob.y + ga[ks][1].z * ob.z + ga[ks][1].w * ob.w;
    mx4.x = fmaxf(mx4.x, fmaxf(amax4(qa[ks][0]), amax4(qa[ks][1])));
    mx4.w = fmaxf(mx4.w, fmaxf(amax4(ga[ks][0]), amax4(ga[ks][1])));
  }
  delta += __shfl_xor(delta, 32, 64);
  // this thread's K / V elements: row pairs x float4 column chunks
  float4 k0[NIT], k1[NIT], v0[NIT], v1[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + 256 * it;
    k0[it] = k1[it] = v0[it] = v1[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < NE) {
      const int kp = e / CH, ch = e - kp * CH;
      const int s0 = rows[2 * kp], s1 = rows[2 * kp + 1];
      if (s0 >= 0) {
        k0[it] = *reinterpret_cast<const float4*>(qkv + (long long)s0 * ld + C + head * D + 4 * ch);
        v0[it] = *reinterpret_cast<const float4*>(qkv + (long long)s0 * ld + 2 * C + head * D + 4 * ch);
      }
      if (s1 >= 0) {
        k1[it] = *reinterpret_cast<const float4*>(qkv + (long long)s1 * ld + C + head * D + 4 * ch);
        v1[it] = *reinterpret_cast<const float4*>(qkv + (long long)s1 * ld + 2 * C + head * D + 4 * ch);
      }
    }
    mx4.y = fmaxf(mx4.y, fmaxf(amax4(k0[it]), amax4(k1[it])));
    mx4.z = fmaxf(mx4.z, fmaxf(amax4(v0[it]), amax4(v1[it])));
  }
  mx4 = bwd_wg_max4(mx4, red);
  float iQ, iK, iV, iG;
  const float sQ = bwd_pow2(mx4.x, iQ), sK = bwd_pow2(mx4.y, iK), sV = bwd_pow2(mx4.z, iV),
              sG = bwd_pow2(mx4.w, iG);
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + 256 * it;
    if (e < NE) {
      const int kp = e / CH, ch = e - kp * CH;
      bwd_stage_pair<D, KD>(Kr, Kt, 2 * kp, ch, k0[it], k1[it], sK);
      bwd_stage_row<KD>(Vr, 2 * kp, ch, v0[it], sV);
      bwd_stage_row<KD>(Vr, 2 * kp + 1, ch, v1[it], sV);
    }
  }
  f16x8 qf[NKS][2], gf[NKS][2];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    bwd_frag(qa[ks][0], qa[ks][1], sQ, qf[ks]);
    bwd_frag(ga[ks][0], ga[ks][1], sG, gf[ks]);
  }
  __syncthreads();

  // S^T[key][query] (log2 units, as the forward: scale * log2(e) folded in)
  floatx16 s[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      f16x8 kf[2];
      bwd_row_frag<KD>(Kr, kb * 32 + l32, 2 * ks + h, kf);
      s[kb] = mfma3<ONE>(kf, qf[ks], s[kb]);
    }
  }
  const float cS = scale * 1.4426950408889634f * iQ * iK;
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      s[kb][r] = key < Kwin ? s[kb][r] * cS : -INFINITY;
      mx = fmaxf(mx, s[kb][r]);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = __builtin_amdgcn_exp2f(s[kb][r] - mx);
      s[kb][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32, 64);
  const float rinv = 1.f / sum;
  if (h == 0 && qown) stats[(long long)qsrc * heads + head] = make_float4(mx, rinv, delta, 0.f);

  // per key block: dP^T = V dO^T, dS^T = P^T (dP^T - Delta), dQ^T += K^T dS^T
  const float cP = iV * iG;
  floatx16 dq;
#pragma unroll
  for (int r = 0; r < 16; ++r) dq[r] = 0.f;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    floatx16 dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      f16x8 vf[2];
      bwd_row_frag<KD>(Vr, kb * 32 + l32, 2 * ks + h, vf);
      dp = mfma3<ONE>(vf, gf[ks], dp);
    }
    float m = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dp[r] = s[kb][r] * rinv * (dp[r] * cP - delta);  // dS^T
      m = fmaxf(m, fabsf(dp[r]));
    }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float isd;
    const float sd = bwd_pow2(m, isd);
    floatx16 t;
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      f16x8 bf[2], kt[2];
      bwd_frag(make_float4(dp[8 * st + 0], dp[8 * st + 1], dp[8 * st + 2], dp[8 * st + 3]),
               make_float4(dp[8 * st + 4], dp[8 * st + 5], dp[8 * st + 6], dp[8 * st + 7]), sd, bf);
      bwd_tr_frag<D>(Kt, l32, 2 * kb + st, h, kt);
      t = mfma3<ONE>(kt, bf, t);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[r] += t[r] * isd;
  }
  if (qown) {
    const float cQ = scale * iK;
    float* dst = dqkv + (long long)qsrc * ld + head * D;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int dd = 8 * g + 4 * h;
      if (dd + 3 < D)
        *reinterpret_cast<float4*>(dst + dd) =
            make_float4(dq[4 * g + 0] * cQ, dq[4 * g + 1] * cQ, dq[4 * g + 2] * cQ, dq[4 * g + 3] * cQ);
    }
  }
}

template <int D, bool ONE = false>
__global__ void __launch_bounds__(256, 3)
window_attn_bwd_kv_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win,
                          int Kwin, int C, float scale, const float* __restrict__ dout, float* __restrict__ dqkv,
                          const float4* __restrict__ stats, int nwin) {
  constexpr int KD = D == 16 ? 16 : 32, NKS = KD / 16, QROW = KD == 16 ? 48 : 64, VST = 136;
  constexpr int RB = 2 * KMAX * QROW, TB = 2 * D * VST * 2;
  constexpr int CH = D / 4, NE = (KMAX / 2) * CH, NIT = (NE + 255) / 256;
  constexpr int DP = D + 4;  // fp32 output staging row stride
  static_assert(2 * KMAX * DP * 4 <= 2 * RB + 2 * TB, "output staging must fit the operand images");
  __shared__ __attribute__((aligned(16))) char lds[2 * RB + 2 * TB];
  __shared__ int rows[KMAX];
  __shared__ float4 stat[KMAX];
  __shared__ float4 red[4];
  char* Qr = lds;
  char* Gr = lds + RB;
  unsigned short* Qt = reinterpret_cast<unsigned short*>(lds + 2 * RB);
  unsigned short* Gt = reinterpret_cast<unsigned short*>(lds + 2 * RB + TB);

  const int heads = C / D;
  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8);
  if (L >= nwin * heads) return;
  const int w = L / heads, head = L - w * heads;
  const int key_start = win[2 * w], query_start = win[2 * w + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  if (tid < KMAX) {
    const int src = tid < Kwin ? order[key_start + tid] : -1;
    rows[tid] = src;
    // queries of this window that another window owns (the ragged last window's padding) or past Kwin: P = 0
    // (exp2(s - inf) = 0, 1/sum = 0) and Delta = 0, exactly as their zero dO in the reference
    stat[tid] = (src >= 0 && key_start + tid >= query_start) ? stats[(long long)src * heads + head]
                                                               : make_float4(INFINITY, 0.f, 0.f, 0.f);
  }
  if (D < KD)
    for (int rr = tid; rr < 4 * KMAX; rr += 256)
      *reinterpret_cast<uint4*>(lds + (rr >> 8) * RB + ((rr >> 7) & 1) * KMAX * QROW + bwd_row_off<KD>(rr & 127, D / 8)) =
          make_uint4(0, 0, 0, 0);
  __syncthreads();
  // this lane's key: k and v slices (B operands of S and dP)
  const int kk = 32 * wid + l32;
  const int ksrc = rows[kk];
  const bool key_ok = ksrc >= 0;
  float4 ka[NKS][2], va[NKS][2];
  float4 mx4 = make_float4(0.f, 0.f, 0.f, 0.f);  // (q, k, v, dO)
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int d0 = 16 * ks + 8 * h;
    const float* base = qkv + (long long)(key_ok ? ksrc : 0) * ld + head * D;
    bwd_load8<D>(base + C, d0, key_ok, ka[ks][0], ka[ks][1]);
    bwd_load8<D>(base + 2 * C, d0, key_ok, va[ks][0], va[ks][1]);
    mx4.y = fmaxf(mx4.y, fmaxf(amax4(ka[ks][0]), amax4(ka[ks][1])));
    mx4.z = fmaxf(mx4.z, fmaxf(amax4(va[ks][0]), amax4(va[ks][1])));
  }
  float4 q0[NIT], q1[NIT], g0[NIT], g1[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + 256 * it;
    q0[it] = q1[it] = g0[it] = g1[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < NE) {
      const int qp = e / CH, ch = e - qp * CH;
      const int r0 = 2 * qp, s0 = rows[r0], s1 = rows[r0 + 1];
      if (s0 >= 0) {
        q0[it] = *reinterpret_cast<const float4*>(qkv + (long long)s0 * ld + head * D + 4 * ch);
        if (key_start + r0 >= query_start)
          g0[it] = *reinterpret_cast<const float4*>(dout + (long long)s0 * C + head * D + 4 * ch);
      }
      if (s1 >= 0) {
        q1[it] = *reinterpret_cast<const float4*>(qkv + (long long)s1 * ld + head * D + 4 * ch);
        if (key_start + r0 + 1 >= query_start)
          g1[it] = *reinterpret_cast<const float4*>(dout + (long long)s1 * C + head * D + 4 * ch);
      }
    }
    mx4.x = fmaxf(mx4.x, fmaxf(amax4(q0[it]), amax4(q1[it])));
    mx4.w = fmaxf(mx4.w, fmaxf(amax4(g0[it]), amax4(g1[it])));
  }
  mx4 = bwd_wg_max4(mx4, red);
  float iQ, iK, iV, iG;
  const float sQ = bwd_pow2(mx4.x, iQ), sK = bwd_pow2(mx4.y, iK), sV = bwd_pow2(mx4.z, iV),
              sG = bwd_pow2(mx4.w, iG);
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + 256 * it;
    if (e < NE) {
      const int qp = e / CH, ch = e - qp * CH;
      bwd_stage_pair<D, KD>(Qr, Qt, 2 * qp, ch, q0[it], q1[it], sQ);
      bwd_stage_pair<D, KD>(Gr, Gt, 2 * qp, ch, g0[it], g1[it], sG);
    }
  }
  f16x8 kf[NKS][2], vf[NKS][2];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    bwd_frag(ka[ks][0], ka[ks][1], sK, kf[ks]);
    bwd_frag(va[ks][0], va[ks][1], sV, vf[ks]);
  }
  __syncthreads();

  const float cS = scale * 1.4426950408889634f * iQ * iK, cP = iG * iV;
  floatx16 dk, dv;
#pragma unroll
  for (int r = 0; r < 16; ++r) dk[r] = dv[r] = 0.f;
#pragma unroll 1
  for (int qb = 0; qb < 4; ++qb) {
    floatx16 sb, pb;
#pragma unroll
    for (int r = 0; r < 16; ++r) sb[r] = pb[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      f16x8 a[2];
      bwd_row_frag<KD>(Qr, qb * 32 + l32, 2 * ks + h, a);
      sb = mfma3<ONE>(a, kf[ks], sb);
      bwd_row_frag<KD>(Gr, qb * 32 + l32, 2 * ks + h, a);
      pb = mfma3<ONE>(a, vf[ks], pb);
    }
    // rows r: query qb*32 + (r&3) + 8(r>>2) + 4h ; P (<= 1) into sb, dS into pb
    float m = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float4 st = stat[qb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h];
      const float P = key_ok ? __builtin_amdgcn_exp2f(sb[r] * cS - st.x) * st.y : 0.f;
      sb[r] = P;
      pb[r] = P * (pb[r] * cP - st.z);
      m = fmaxf(m, fabsf(pb[r]));
    }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float isd;
    const float sd = bwd_pow2(m, isd);
    floatx16 t;
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      f16x8 bp[2], bd[2], at[2];
      bwd_frag(make_float4(sb[8 * st + 0], sb[8 * st + 1], sb[8 * st + 2], sb[8 * st + 3]),
               make_float4(sb[8 * st + 4], sb[8 * st + 5], sb[8 * st + 6], sb[8 * st + 7]), 16384.f, bp);
      bwd_tr_frag<D>(Gt, l32, 2 * qb + st, h, at);
      dv = mfma3<ONE>(at, bp, dv);
      bwd_frag(make_float4(pb[8 * st + 0], pb[8 * st + 1], pb[8 * st + 2], pb[8 * st + 3]),
               make_float4(pb[8 * st + 4], pb[8 * st + 5], pb[8 * st + 6], pb[8 * st + 7]), sd, bd);
      bwd_tr_frag<D>(Qt, l32, 2 * qb + st, h, at);
      t = mfma3<ONE>(at, bd, t);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[r] += t[r] * isd;
  }
  // dK / dV leave through LDS (whole row segments per store); keys shared with the neighbouring window (the ragged
  // last window's overlap) are added atomically, every other key is owned by this window and stored plainly
  const float cK = scale * iQ, cV = iG * (1.f / 16384.f);
  __syncthreads();  // all waves done with the operand images
  float* Ok = reinterpret_cast<float*>(lds);
  float* Ov = Ok + KMAX * DP;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int dd = (r & 3) + 8 * (r >> 2) + 4 * h;
    if (dd < D) {
      Ok[kk * DP + dd] = dk[r] * cK;
      Ov[kk * DP + dd] = dv[r] * cV;
    }
  }
  __syncthreads();
  const int next_ks = (w + 1 < nwin) ? win[2 * (w + 1)] : 0x7fffffff;
  for (int e = tid; e < Kwin * 2 * CH; e += 256) {
    const int row = e / (2 * CH);
    const int rem = e - row * 2 * CH;
    const int mat = rem / CH, ch = rem - mat * CH;
    const float4 v = *reinterpret_cast<const float4*>(&(mat == 0 ? Ok : Ov)[row * DP + 4 * ch]);
    float* dst = dqkv + (long long)rows[row] * ld + (mat + 1) * C + head * D + 4 * ch;
    const int pos = key_start + row;
    if (pos < query_start || pos >= next_ks) {
      atomicAdd(dst + 0, v.x);
      atomicAdd(dst + 1, v.y);
      atomicAdd(dst + 2, v.z);
      atomicAdd(dst + 3, v.w);
    } else {
      *reinterpret_cast<float4*>(dst) = v;
    }
  }
}

// SFX_ATTN_SEQ=1: the pipelined kernel (window_attn_seq_kernel) on at most 512 workgroups, SFX_ATTN_SEQ=<n>
// (n > 1) on at most n; default and 0: one (window, head) item per workgroup (window_attn_split_kernel), which
// measured faster (config B 568 vs 553 renders/s at 768 / 1024 workgroups, profiles/r04_ab_bench.txt)
int attn_seq() {
  const char* e = getenv("SFX_ATTN_SEQ");  // (read per call: tests switch it)
  if (!e || !e[0]) return 0;
  const int v = atoi(e);
  return v == 0 ? 0 : v > 1 ? v : 512;
}

}  // namespace

extern "C" {

// qkv [N, 3C] (point order), order [N] serialized->point, win [num_windows][2], out [N, C]
int sfx_window_attention(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                         const int* order, const int* win, float scale, float* out,
                         const unsigned long long* qkv_amax, unsigned qkv_tag, void* stream) {
  SFX_REQUIRE(num_windows >= 0, "sfx_window_attention: num_windows < 0");
  SFX_REQUIRE(window >= 1 && window <= KMAX, "sfx_window_attention: window must be in [1, 128]");
  SFX_REQUIRE(heads * head_dim == channels, "sfx_window_attention: heads * head_dim != channels");
  SFX_REQUIRE(head_dim == 16 || head_dim == 24 || head_dim == 32,
              "sfx_window_attention: head_dim %d unsupported (16, 24, 32)", head_dim);
  if (num_windows == 0) return SFX_OK;
  SFX_REQUIRE(qkv && order && win && out, "sfx_window_attention: null buffer");
  dim3 grid(num_windows, heads);
  const long long nblk = ((long long)num_windows * heads + 7) / 8 * 8;
  SFX_REQUIRE(nblk < (1ll << 31), "sfx_window_attention: too many windows");
  hipStream_t st = sfx::as_stream(stream);
  static int exact = -1;  // SFX_ATTN_PREC=fp32: the v_mfma_f32_32x32x2_f32 kernel
  if (exact < 0) {
    const char* e = getenv("SFX_ATTN_PREC");
    exact = (e && e[0] == 'f') ? 1 : 0;
  }
  if (exact) {
    if (head_dim == 16)
      window_attn_kernel<16><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, out);
    else if (head_dim == 24)
      window_attn_kernel<24><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, out);
    else
      window_attn_kernel<32><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, out);
  } else if (const int seq_wgs = qkv_amax ? attn_seq() : 0) {  // fp16x2 terms, pipelined over (window, head) items
    const int items = num_windows * heads;
    const int ipw = (items + seq_wgs - 1) / seq_wgs;  // at most seq_wgs workgroups (512: one round at 2 per CU)
    const long long nwg = ((long long)(items + ipw - 1) / ipw + 7) / 8 * 8;
#define SFX_ATTN_SEQ(DD)                                                                                     \
  window_attn_seq_kernel<DD><<<dim3((unsigned)nwg), 256, 0, st>>>(qkv, order, win, window, channels, scale, out, \
                                                                   qkv_amax, qkv_tag, items, ipw)
    if (head_dim == 16) SFX_ATTN_SEQ(16);
    else if (head_dim == 24) SFX_ATTN_SEQ(24);
    else SFX_ATTN_SEQ(32);
#undef SFX_ATTN_SEQ
  } else if (qkv_amax) {  // fp16x2 terms (the caller bounds |qkv|)
#define SFX_ATTN(DD, F, O)                                                                                  \
  window_attn_split_kernel<DD, F, O><<<dim3((unsigned)nblk), 256, 0, st>>>(qkv, order, win, window, channels, scale, \
                                                                           out, qkv_amax, qkv_tag, num_windows)
    if (sfx_get_precision() == 1) {  // reference-precision mode: single fp16 products
      if (head_dim == 16) SFX_ATTN(16, true, true);
      else if (head_dim == 24) SFX_ATTN(24, true, true);
      else SFX_ATTN(32, true, true);
    } else if (head_dim == 16) SFX_ATTN(16, true, false);
    else if (head_dim == 24) SFX_ATTN(24, true, false);
    else SFX_ATTN(32, true, false);
  } else {
    if (sfx_get_precision() == 1) {
      if (head_dim == 16) SFX_ATTN(16, false, true);
      else if (head_dim == 24) SFX_ATTN(24, false, true);
      else SFX_ATTN(32, false, true);
    } else if (head_dim == 16) SFX_ATTN(16, false, false);
    else if (head_dim == 24) SFX_ATTN(24, false, false);
    else SFX_ATTN(32, false, false);
#undef SFX_ATTN
  }
  return sfx::check_launch("sfx_window_attention");
}

// flash mode: win3 [num_windows][3] = (key_start, query_start, key_count), key_count <= max_window
int sfx_window_attention_varlen(int num_windows, int max_window, int heads, int head_dim, int channels,
                                const float* qkv, const int* order, const int* win3, float scale, float* out,
                                const unsigned long long* qkv_amax, unsigned qkv_tag, void* stream) {
  SFX_REQUIRE(num_windows >= 0, "sfx_window_attention_varlen: num_windows < 0");
  SFX_REQUIRE(max_window >= 1 && max_window <= (1 << 20), "sfx_window_attention_varlen: max_window out of [1, 2^20]");
  SFX_REQUIRE(heads * head_dim == channels, "sfx_window_attention_varlen: heads * head_dim != channels");
  SFX_REQUIRE(head_dim == 16 || head_dim == 24 || head_dim == 32,
              "sfx_window_attention_varlen: head_dim %d unsupported (16, 24, 32)", head_dim);
  if (num_windows == 0) return SFX_OK;
  SFX_REQUIRE(qkv && order && win3 && out, "sfx_window_attention_varlen: null buffer");
  const int qblocks = (max_window + KMAX - 1) / KMAX;
  const long long nblk = ((long long)num_windows * qblocks * heads + 7) / 8 * 8;
  SFX_REQUIRE(nblk < (1ll << 31) && heads <= 65535, "sfx_window_attention_varlen: grid too large");
  hipStream_t st = sfx::as_stream(stream);
  static int exact = -1;  // SFX_ATTN_PREC=fp32: the v_mfma_f32_32x32x2_f32 kernel
  if (exact < 0) {
    const char* e = getenv("SFX_ATTN_PREC");
    exact = (e && e[0] == 'f') ? 1 : 0;
  }
  if (exact) {
    dim3 grid((unsigned)(num_windows * qblocks), heads);
    if (head_dim == 16)
      window_attn_flash_kernel<16><<<grid, 256, 0, st>>>(qkv, order, win3, qblocks, channels, scale, out);
    else if (head_dim == 24)
      window_attn_flash_kernel<24><<<grid, 256, 0, st>>>(qkv, order, win3, qblocks, channels, scale, out);
    else
      window_attn_flash_kernel<32><<<grid, 256, 0, st>>>(qkv, order, win3, qblocks, channels, scale, out);
    return sfx::check_launch("sfx_window_attention_varlen");
  }
#define SFX_ATTN(DD, F)                                                                                       \
  window_attn_split_flash_kernel<DD, F><<<dim3((unsigned)nblk), 256, 0, st>>>(qkv, order, win3, qblocks, channels, \
                                                                              scale, out, qkv_amax, qkv_tag,   \
                                                                              num_windows)
  if (qkv_amax) {  // fp16x2 terms (the caller bounds |qkv|)
    if (head_dim == 16) SFX_ATTN(16, true);
    else if (head_dim == 24) SFX_ATTN(24, true);
    else SFX_ATTN(32, true);
  } else {
    if (head_dim == 16) SFX_ATTN(16, false);
    else if (head_dim == 24) SFX_ATTN(24, false);
    else SFX_ATTN(32, false);
  }
#undef SFX_ATTN
  return sfx::check_launch("sfx_window_attention_varlen");
}

// flash-mode backward: dqkv [N, 3C] zero-filled by the caller, stats [N][heads][2] floats of workspace
int sfx_window_attention_varlen_bwd(int num_windows, int max_window, int heads, int head_dim, int channels,
                                    const float* qkv, const int* order, const int* win3, float scale,
                                    const float* dout, float* dqkv, float* stats, void* stream) {
  SFX_REQUIRE(num_windows >= 0, "sfx_window_attention_varlen_bwd: num_windows < 0");
  SFX_REQUIRE(max_window >= 1 && max_window <= (1 << 20),
              "sfx_window_attention_varlen_bwd: max_window out of [1, 2^20]");
  SFX_REQUIRE(heads * head_dim == channels, "sfx_window_attention_varlen_bwd: heads * head_dim != channels");
  SFX_REQUIRE(head_dim == 16 || head_dim == 24 || head_dim == 32,
              "sfx_window_attention_varlen_bwd: head_dim %d unsupported (16, 24, 32)", head_dim);
  if (num_windows == 0) return SFX_OK;
  SFX_REQUIRE(qkv && order && win3 && dout && dqkv && stats, "sfx_window_attention_varlen_bwd: null buffer");
  const int blocks = (max_window + FB - 1) / FB;
  SFX_REQUIRE((long long)num_windows * blocks < (1ll << 31) && heads <= 65535,
              "sfx_window_attention_varlen_bwd: grid too large");
  dim3 grid((unsigned)(num_windows * blocks), heads);
  hipStream_t st = sfx::as_stream(stream);
#define SFX_FBWD(DD)                                                                                           \
  do {                                                                                                         \
    flash_bwd_query_kernel<DD><<<grid, FB, 0, st>>>(qkv, order, win3, blocks, channels, heads, scale, dout, dqkv, \
                                                     stats);                                                   \
    flash_bwd_key_kernel<DD><<<grid, FB, 0, st>>>(qkv, order, win3, blocks, channels, heads, scale, dout, dqkv, \
                                                   stats);                                                     \
  } while (0)
  if (head_dim == 16) SFX_FBWD(16);
  else if (head_dim == 24) SFX_FBWD(24);
  else SFX_FBWD(32);
#undef SFX_FBWD
  return sfx::check_launch("sfx_window_attention_varlen_bwd");
}

// dout [N, C] = d(attention output); attn_out [N, C] = the forward's output; dqkv [N, 3C] (every element written;
// the exact kernel needs it zero-filled by the caller); stats: workspace of N * heads float4 (query pass -> key
// pass).  SFX_ATTN_PREC=fp32: the exact single-kernel backward (attn_out and stats unused, dqkv zero-filled)
int sfx_window_attention_bwd(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                             const int* order, const int* win, float scale, const float* attn_out, const float* dout,
                             float* dqkv, float* stats, void* stream) {
  SFX_REQUIRE(num_windows >= 0, "sfx_window_attention_bwd: num_windows < 0");
  SFX_REQUIRE(window >= 1 && window <= KMAX, "sfx_window_attention_bwd: window must be in [1, 128]");
  SFX_REQUIRE(heads * head_dim == channels, "sfx_window_attention_bwd: heads * head_dim != channels");
  SFX_REQUIRE(head_dim == 16 || head_dim == 24 || head_dim == 32,
              "sfx_window_attention_bwd: head_dim %d unsupported (16, 24, 32)", head_dim);
  if (num_windows == 0) return SFX_OK;
  SFX_REQUIRE(qkv && order && win && dout && dqkv, "sfx_window_attention_bwd: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  static int exact = -1;
  if (exact < 0) {
    const char* e = getenv("SFX_ATTN_PREC");
    exact = (e && e[0] == 'f') ? 1 : 0;
  }
  if (!exact) {
    SFX_REQUIRE(attn_out && stats, "sfx_window_attention_bwd: null attn_out / stats");
    const long long nblk = ((long long)num_windows * heads + 7) / 8 * 8;
    SFX_REQUIRE(nblk < (1ll << 31), "sfx_window_attention_bwd: too many windows");
    float4* st4 = reinterpret_cast<float4*>(stats);
#define SFX_ABWD(DD, ONE)                                                                                         \
  do {                                                                                                            \
    window_attn_bwd_q_kernel<DD, ONE><<<dim3((unsigned)nblk), 256, 0, st>>>(qkv, order, win, window, channels,    \
                                                                            scale, attn_out, dout, dqkv, st4,    \
                                                                            num_windows);                         \
    window_attn_bwd_kv_kernel<DD, ONE><<<dim3((unsigned)nblk), 256, 0, st>>>(qkv, order, win, window, channels,   \
                                                                             scale, dout, dqkv, st4, num_windows); \
  } while (0)
    const bool one = sfx_get_precision() == 1;  // reference-precision mode: single fp16 products
    if (head_dim == 16) { if (one) SFX_ABWD(16, true); else SFX_ABWD(16, false); }
    else if (head_dim == 24) { if (one) SFX_ABWD(24, true); else SFX_ABWD(24, false); }
    else { if (one) SFX_ABWD(32, true); else SFX_ABWD(32, false); }
#undef SFX_ABWD
    return sfx::check_launch("sfx_window_attention_bwd");
  }
  dim3 grid(num_windows, heads);
  if (head_dim == 16)
    window_attn_bwd_kernel<16><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, dout, dqkv);
  else if (head_dim == 24)
    window_attn_bwd_kernel<24><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, dout, dqkv);
  else
    window_attn_bwd_kernel<32><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, dout, dqkv);
  return sfx::check_launch("sfx_window_attention_bwd");
}

}  // extern "C"
