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
#include "common.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int KMAX = 128;

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

}  // namespace

extern "C" {

// qkv [N, 3C] (point order), order [N] serialized->point, win [num_windows][2], out [N, C]
int sfx_window_attention(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                         const int* order, const int* win, float scale, float* out, void* stream) {
  SFX_REQUIRE(num_windows >= 0, "sfx_window_attention: num_windows < 0");
  SFX_REQUIRE(window >= 1 && window <= KMAX, "sfx_window_attention: window must be in [1, 128]");
  SFX_REQUIRE(heads * head_dim == channels, "sfx_window_attention: heads * head_dim != channels");
  SFX_REQUIRE(head_dim == 16 || head_dim == 24 || head_dim == 32,
              "sfx_window_attention: head_dim %d unsupported (16, 24, 32)", head_dim);
  if (num_windows == 0) return SFX_OK;
  SFX_REQUIRE(qkv && order && win && out, "sfx_window_attention: null buffer");
  dim3 grid(num_windows, heads);
  hipStream_t st = sfx::as_stream(stream);
  if (head_dim == 16)
    window_attn_kernel<16><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, out);
  else if (head_dim == 24)
    window_attn_kernel<24><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, out);
  else
    window_attn_kernel<32><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, out);
  return sfx::check_launch("sfx_window_attention");
}

// dout [N, C] = d(attention output); dqkv [N, 3C] zero-filled by the caller (dK/dV accumulate)
int sfx_window_attention_bwd(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                             const int* order, const int* win, float scale, const float* dout, float* dqkv,
                             void* stream) {
  SFX_REQUIRE(num_windows >= 0, "sfx_window_attention_bwd: num_windows < 0");
  SFX_REQUIRE(window >= 1 && window <= KMAX, "sfx_window_attention_bwd: window must be in [1, 128]");
  SFX_REQUIRE(heads * head_dim == channels, "sfx_window_attention_bwd: heads * head_dim != channels");
  SFX_REQUIRE(head_dim == 16 || head_dim == 24 || head_dim == 32,
              "sfx_window_attention_bwd: head_dim %d unsupported (16, 24, 32)", head_dim);
  if (num_windows == 0) return SFX_OK;
  SFX_REQUIRE(qkv && order && win && dout && dqkv, "sfx_window_attention_bwd: null buffer");
  dim3 grid(num_windows, heads);
  hipStream_t st = sfx::as_stream(stream);
  if (head_dim == 16)
    window_attn_bwd_kernel<16><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, dout, dqkv);
  else if (head_dim == 24)
    window_attn_bwd_kernel<24><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, dout, dqkv);
  else
    window_attn_bwd_kernel<32><<<grid, 256, 0, st>>>(qkv, order, win, window, channels, scale, dout, dqkv);
  return sfx::check_launch("sfx_window_attention_bwd");
}

}  // extern "C"
