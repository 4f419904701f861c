// Serialized windowed attention fused with the attention's output projection and the Block's residual add:
//
//   x2[row] = x1[row] + proj_b + proj_W . concat_heads( softmax(q k^T * scale) v )[row]
//
// (PTv3 Block, restated at calflops.py:51-69: `feat = shortcut + drop_path(attn(norm1(feat)))` with
// SerializedAttention.proj the last op of attn; attention math visualize.py:140-179; reference
// models/pointtransformer_v3.py:121-126, patch 128, non-flash).  The per-head outputs never leave the chip: the
// attention output (N x C fp32) is neither written nor re-read by a projection GEMM, and one launch replaces the
// attention launch + the projection GEMM launch of window_attn_split_kernel + gemm_kernel.
//
// gfx950 mapping (the split kernel's dataflow, attention.hip, per head, with every head of a window in ONE
// workgroup so the projection can sum over heads in registers):
//   * workgroup = one window (NWV = 4 waves, 128 queries) or half of one (NWV = 2, 64 queries), wave = 32 queries on
//     the lanes; the window's keys (128) are staged per head into LDS as fp16x2 term images: K [key][dd],
//     V^T [dd][key] (as window_attn_split_kernel<D, true>), and the head's projection slice Wp[:, head] [cout][dd]
//     from the weight's pre-split (sfx_weight_split: per-row power-of-two scale, fp16 h / l terms);
//   * S^T = K Q^T (query on the lane column, keys in registers), register softmax (exp2, log2 e folded into q),
//     O^T = V^T P^T with P^T straight from the softmax registers;
//   * O^T's accumulator rows (dd) are the k index of the projection: Y^T[cout][q] += Wp_h[cout][dd] O^T[dd][q]
//     takes O^T from registers with no LDS round trip (the 32x32 C layout's permuted k order: element j of lane
//     half h of k-step s is dd = 16 s + 8 (j >> 2) + 4 h + (j & 3), the Wp image is staged in that order), C / 32
//     accumulator blocks of 32 couts x 32 queries per wave, summed over the heads;
//   * epilogue: Y / (row scale of Wp x qkv scale) + bias + x1 -> x2, 16-byte row stores through the serialized order.
// Operand scales: q, k, v and O (a convex combination of v rows: |O| <= max |v|) by the power of two that puts the
// qkv bound (amax slot) in [2^14, 2^15); probabilities (0, 1] by 2^14; Wp rows by their own power of two.  Every
// product is h*h + h*l + l*h on v_mfma_f32_32x32x16_f16 with fp32 accumulation: fp32-level accuracy (the split
// kernel's argument), so the refine keeps its 1e-5 bar.
#include <cstdlib>

#include "common.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));

constexpr int KMAX = 128;

// V^T chunk swizzle (attention.hip vt_swz): chunk c of V^T row dd at c ^ 2 parity(dd >> 2)
__device__ __forceinline__ int vt_swz(int dd) { return (__builtin_popcount((unsigned)(dd >> 2)) & 1) << 1; }

__device__ __forceinline__ floatx16 mfma16(const f16x8& a, const f16x8& b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int D, int C, int NWV>
__global__ void __launch_bounds__(NWV * 64, 8 / NWV)
attn_proj_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win, int Kwin,
                 float scale, const unsigned long long* __restrict__ qkv_amax, unsigned qkv_tag,
                 const uint4* __restrict__ wsp, const float* __restrict__ winv, const float* __restrict__ bias,
                 const float* __restrict__ x1, long long ldx1, float* __restrict__ x2, long long ldx2, int nwin) {
  constexpr int H = C / D;
  constexpr int KD = D == 16 ? 16 : 32;  // K image / q fragment depth (S^T contraction, zero past D)
  constexpr int NKS = KD / 16;
  constexpr int QROW = KD == 16 ? 48 : 64;  // bytes per K term row
  constexpr int VST = 136;                  // V^T row stride (16-bit elements)
  constexpr int KB = 2 * KMAX * QROW;
  constexpr int VB = 2 * D * VST * 2;
  constexpr int NKP = (D + 15) / 16;  // projection k-steps over the head's dd
  constexpr int WROW = NKP * 32;      // Wp image bytes per cout row and term (NKP steps x 2 lane halves x 16 B)
  constexpr int WB = 2 * C * WROW;
  constexpr int NCB = C / 32;         // 32-cout accumulator blocks
  constexpr int NT = NWV * 64;
  constexpr int QPW = NWV * 32;       // queries per workgroup
  constexpr int QS = KMAX / QPW;      // workgroups per window
  constexpr int CH = D / 4;           // float4 per head row slice
  static_assert(C % 32 == 0 && C % D == 0, "shape");

  // operand scales: qkv (and O) by sq, probabilities by 2^14
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

  __shared__ __attribute__((aligned(16))) char lds[KB + VB + WB];
  __shared__ int rows[KMAX];
  char* Ks = lds;
  unsigned short* Vt = reinterpret_cast<unsigned short*>(lds + KB);
  char* Ws = lds + KB + VB;
  auto qk_off = [](int r, int c) -> int {
    return KD == 16 ? r * 48 + c * 16 : r * 64 + (((c ^ (r >> 2)) & 3) << 4);
  };

  // XCD-aware numbering (as window_attn_split_kernel): the QS workgroups of a window run back to back on one XCD
  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8);
  if (L >= nwin * QS) return;
  const int w = L / QS, qh = L - w * QS;
  const int key_start = win[2 * w], query_start = win[2 * w + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const long long ld = 3ll * C;

  for (int r = tid; r < KMAX; r += NT) rows[r] = r < Kwin ? order[key_start + r] : -1;
  if (D < KD)  // K columns D..KD-1: zero once, the per-head staging never writes them
    for (int rr = tid; rr < 2 * KMAX; rr += NT) *reinterpret_cast<uint4*>(Ks + qk_off(rr, D / 8)) = make_uint4(0, 0, 0, 0);
  __syncthreads();

  const int qi = QPW * qh + 32 * wid + l32;  // this lane's query (window position)
  const int qrow = rows[qi];
  floatx16 y[NCB];
#pragma unroll
  for (int b = 0; b < NCB; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) y[b][r] = 0.f;

#pragma unroll 1
  for (int hd = 0; hd < H; ++hd) {
    if (hd) __syncthreads();  // every wave is done reading the previous head's images
    // ---- stage K_h [key][dd], V_h^T [dd][key] and Wp_h [cout][dd] (fp16x2 terms) ----
    for (int e = tid; e < KMAX * CH; e += NT) {
      const int row = e / CH, ch = e - row * CH;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int src = rows[row];
      if (src >= 0) v = *reinterpret_cast<const float4*>(qkv + (long long)src * ld + C + hd * D + 4 * ch);
      uint2 t[2];
      sfx::split2h(v, sq, t);
      const int o = qk_off(row, ch >> 1) + ((ch & 1) << 3);
      *reinterpret_cast<uint2*>(Ks + o) = t[0];
      *reinterpret_cast<uint2*>(Ks + KMAX * QROW + o) = t[1];
    }
    for (int e = tid; e < (KMAX / 2) * CH; e += NT) {
      const int kp = e / CH, ch = e - kp * CH;
      const int row = 2 * kp;
      const int s0 = rows[row], s1 = rows[row + 1];
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
      if (s0 >= 0) v0 = *reinterpret_cast<const float4*>(qkv + (long long)s0 * ld + 2 * C + hd * D + 4 * ch);
      if (s1 >= 0) v1 = *reinterpret_cast<const float4*>(qkv + (long long)s1 * ld + 2 * C + hd * D + 4 * ch);
      uint2 t0[2], t1[2];
      sfx::split2h(v0, sq, t0);
      sfx::split2h(v1, sq, t1);
      const int kk = row & 15;  // even: keys row, row + 1 land on adjacent positions
      const int pos = (row & ~15) + 8 * ((kk >> 2) & 1) + (((kk >> 3) << 2) | (kk & 3));
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        unsigned* vt = reinterpret_cast<unsigned*>(Vt + (q * D + 4 * ch) * VST + (pos ^ (8 * vt_swz(4 * ch))));
        vt[0] = (t0[q].x & 0xffffu) | (t1[q].x << 16);
        vt[VST / 2] = (t0[q].x >> 16) | (t1[q].x & 0xffff0000u);
        vt[VST] = (t0[q].y & 0xffffu) | (t1[q].y << 16);
        vt[3 * VST / 2] = (t0[q].y >> 16) | (t1[q].y & 0xffff0000u);
      }
    }
    // Wp_h: chunk c = 2 s + half of cout row n holds the dd of k-step s, lane half `half` in the MFMA's permuted
    // order: 4-element groups g0 = 4 s + half (dd 16 s + 4 half ..) and g1 = g0 + 2 (dd 16 s + 8 + 4 half ..); a group
    // of the pre-split is 16 bytes (4 fp16 h terms, then 4 fp16 l terms); groups at dd >= D are zero
    for (int e = tid; e < C * 2 * NKP; e += NT) {
      const int n = e / (2 * NKP), c = e - n * (2 * NKP);
      const int g0 = 4 * (c >> 1) + (c & 1), g1 = g0 + 2;
      uint4 a = make_uint4(0, 0, 0, 0), b = a;
      const uint4* wr = wsp + (long long)n * (C / 4) + hd * (D / 4);
      if (4 * g0 < D) a = wr[g0];
      if (4 * g1 < D) b = wr[g1];
      *reinterpret_cast<uint4*>(Ws + n * WROW + c * 16) = make_uint4(a.x, a.y, b.x, b.y);
      *reinterpret_cast<uint4*>(Ws + C * WROW + n * WROW + c * 16) = make_uint4(a.z, a.w, b.z, b.w);
    }
    // this lane's query slices (B operand of S^T = K Q^T): dd = 16 ks + 8 h + j, zero past D
    f16x8 qf[NKS][2];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = 16 * ks + 8 * h;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (qrow >= 0 && d0 < D) {
        const float* qp = qkv + (long long)qrow * ld + hd * D + d0;
        a = *reinterpret_cast<const float4*>(qp);
        if (d0 + 4 < D) b = *reinterpret_cast<const float4*>(qp + 4);
      }
      const float qs = scale * 1.4426950408889634f;  // scale * log2(e): the exponentials are plain exp2
      a.x *= qs; a.y *= qs; a.z *= qs; a.w *= qs;
      b.x *= qs; b.y *= qs; b.z *= qs; b.w *= qs;
      uint2 ta[2], tb[2];
      sfx::split2h(a, sq, ta);
      sfx::split2h(b, sq, tb);
#pragma unroll
      for (int q = 0; q < 2; ++q) qf[ks][q] = __builtin_bit_cast(f16x8, (uintx4){ta[q].x, ta[q].y, tb[q].x, tb[q].y});
    }
    __syncthreads();

    // ---- S^T[key][query] (4 key blocks of 32), three term products each, smallest first ----
    floatx16 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int o = qk_off(kb * 32 + l32, 2 * ks + h);
        const f16x8 kh = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(Ks + o));
        const f16x8 kl = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(Ks + KMAX * QROW + o));
        s[kb] = mfma16(kl, qf[ks][0], s[kb]);
        s[kb] = mfma16(kh, qf[ks][1], s[kb]);
        s[kb] = mfma16(kh, qf[ks][0], s[kb]);
      }
    const float iqq = iq * iq;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kb][r] *= iqq;
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
        const float ex = __builtin_amdgcn_exp2f(s[kb][r] - mx);
        s[kb][r] = ex;
        sum += ex;
      }
    sum += __shfl_xor(sum, 32, 64);
    const float rinv = 1.f / sum;

    // ---- O^T[dd][query] = V^T P^T (P^T from the softmax registers, scaled by 2^14) ----
    floatx16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        uint2 a[2], b[2];
        sfx::split2h(make_float4(s[kb][8 * st + 0], s[kb][8 * st + 1], s[kb][8 * st + 2], s[kb][8 * st + 3]), 16384.f, a);
        sfx::split2h(make_float4(s[kb][8 * st + 4], s[kb][8 * st + 5], s[kb][8 * st + 6], s[kb][8 * st + 7]), 16384.f, b);
        const f16x8 ph = __builtin_bit_cast(f16x8, make_uint4(a[0].x, a[0].y, b[0].x, b[0].y));
        const f16x8 pl = __builtin_bit_cast(f16x8, make_uint4(a[1].x, a[1].y, b[1].x, b[1].y));
        uint4 vh = make_uint4(0, 0, 0, 0), vl = vh;  // dd = l32 >= D: zero rows of V^T
        if (l32 < D) {
          const int co = ((2 * (2 * kb + st) + h) ^ vt_swz(l32)) << 3;
          vh = *reinterpret_cast<const uint4*>(Vt + l32 * VST + co);
          vl = *reinterpret_cast<const uint4*>(Vt + (D + l32) * VST + co);
        }
        const f16x8 fvh = __builtin_bit_cast(f16x8, vh), fvl = __builtin_bit_cast(f16x8, vl);
        o = mfma16(fvl, ph, o);
        o = mfma16(fvh, pl, o);
        o = mfma16(fvh, ph, o);
      }

    // ---- Y^T[cout][query] += Wp_h O_h^T: O^T (true values x sq) split into fp16 terms, registers 8s..8s+7 as the
    // B fragment of k-step s (rows dd >= D are zero: V^T rows past D fed zeros) ----
    const float osc = rinv * (1.f / 16384.f);  // o = 2^14 sq sum_k p v  ->  O sq
    f16x8 oh[NKP], ol[NKP];
#pragma unroll
    for (int sp = 0; sp < NKP; ++sp) {
      uint2 a[2], b[2];
      sfx::split2h(make_float4(o[8 * sp + 0], o[8 * sp + 1], o[8 * sp + 2], o[8 * sp + 3]), osc, a);
      sfx::split2h(make_float4(o[8 * sp + 4], o[8 * sp + 5], o[8 * sp + 6], o[8 * sp + 7]), osc, b);
      oh[sp] = __builtin_bit_cast(f16x8, make_uint4(a[0].x, a[0].y, b[0].x, b[0].y));
      ol[sp] = __builtin_bit_cast(f16x8, make_uint4(a[1].x, a[1].y, b[1].x, b[1].y));
    }
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int sp = 0; sp < NKP; ++sp) {
        const int wo = (cb * 32 + l32) * WROW + (2 * sp + h) * 16;
        const f16x8 wh = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(Ws + wo));
        const f16x8 wl = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(Ws + C * WROW + wo));
        y[cb] = mfma16(wl, oh[sp], y[cb]);
        y[cb] = mfma16(wh, ol[sp], y[cb]);
        y[cb] = mfma16(wh, oh[sp], y[cb]);
      }
  }

  // ---- epilogue: x2 = Y / (s_w sq) + b + x1, lane = query, 4 consecutive couts per register group ----
  if (qi < Kwin && key_start + qi >= query_start) {
    const float* xr = x1 + (long long)qrow * ldx1;
    float* dst = x2 + (long long)qrow * ldx2;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n0 = cb * 32 + 8 * g + 4 * h;
        const float4 wi = *reinterpret_cast<const float4*>(winv + n0);
        const float4 bb = *reinterpret_cast<const float4*>(bias + n0);
        const float4 xx = *reinterpret_cast<const float4*>(xr + n0);
        float4 r;
        r.x = y[cb][4 * g + 0] * (wi.x * iq) + bb.x + xx.x;
        r.y = y[cb][4 * g + 1] * (wi.y * iq) + bb.y + xx.y;
        r.z = y[cb][4 * g + 2] * (wi.z * iq) + bb.z + xx.z;
        r.w = y[cb][4 * g + 3] * (wi.w * iq) + bb.w + xx.w;
        *reinterpret_cast<float4*>(dst + n0) = r;
      }
  }
}

template <int D, int C, int NWV>
void launch(int nwin, int K, const float* qkv, const int* order, const int* win, float scale,
            const unsigned long long* amax, unsigned tag, const float* wsp, const float* winv, const float* bias,
            const float* x1, long long ldx1, float* x2, long long ldx2, hipStream_t st) {
  constexpr int QS = KMAX / (32 * NWV);
  const long long nblk = ((long long)nwin * QS + 7) / 8 * 8;
  attn_proj_kernel<D, C, NWV><<<dim3((unsigned)nblk), NWV * 64, 0, st>>>(
      qkv, order, win, K, scale, amax, tag, reinterpret_cast<const uint4*>(wsp), winv, bias, x1, ldx1, x2, ldx2, nwin);
}

// workgroup size: 2 waves (half a window) when one-window workgroups would leave most of the chip's
// workgroup slots empty (SFX_ATTN_PROJ_WAVES = 2 / 4 forces)
int proj_waves(int nwin, int C) {
  static int force = -1;
  if (force < 0) {
    const char* e = getenv("SFX_ATTN_PROJ_WAVES");
    force = (e && *e) ? atoi(e) : 0;
  }
  if (force == 2 || force == 4) return force;
  (void)C;
  return nwin < 512 ? 2 : 4;
}

}  // namespace

extern "C" {

// (ABI v15) x2 = x1 + proj(attention(qkv)) for the non-flash windows (sfx_window_attention's table and scale)
int sfx_window_attention_proj(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                              const int* order, const int* win, float scale, const unsigned long long* qkv_amax,
                              unsigned qkv_tag, const float* w_split, const float* w_inv, const float* bias,
                              const float* x1, long long ldx1, float* x2, long long ldx2, void* stream) {
  SFX_REQUIRE(num_windows >= 0, "sfx_window_attention_proj: num_windows < 0");
  SFX_REQUIRE(window >= 1 && window <= KMAX, "sfx_window_attention_proj: window must be in [1, 128]");
  SFX_REQUIRE(heads * head_dim == channels, "sfx_window_attention_proj: heads * head_dim != channels");
  const bool shape_ok = (head_dim == 32 && channels == 64) || (head_dim == 24 && channels == 96) ||
                        (head_dim == 16 && (channels == 128 || channels == 256));
  SFX_REQUIRE(shape_ok, "sfx_window_attention_proj: (head_dim %d, channels %d) unsupported ((32, 64), (24, 96), "
              "(16, 128), (16, 256))", head_dim, channels);
  if (num_windows == 0) return SFX_OK;
  SFX_REQUIRE(qkv && order && win && qkv_amax && w_split && w_inv && bias && x1 && x2,
              "sfx_window_attention_proj: null buffer");
  SFX_REQUIRE(ldx1 >= channels && ldx2 >= channels && ldx1 % 4 == 0 && ldx2 % 4 == 0,
              "sfx_window_attention_proj: leading dimensions");
  SFX_REQUIRE(((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(w_split) |
                reinterpret_cast<uintptr_t>(w_inv) | reinterpret_cast<uintptr_t>(bias) |
                reinterpret_cast<uintptr_t>(x1) | reinterpret_cast<uintptr_t>(x2)) & 15) == 0,
              "sfx_window_attention_proj: buffers must be 16-byte aligned");
  SFX_REQUIRE(x1 != x2, "sfx_window_attention_proj: in-place output is not supported");
  SFX_REQUIRE((long long)num_windows * 2 < (1ll << 31), "sfx_window_attention_proj: too many windows");
  hipStream_t st = sfx::as_stream(stream);
  const int nwv = proj_waves(num_windows, channels);
#define SFX_AP(DD, CC)                                                                                            \
  (nwv == 2 ? launch<DD, CC, 2>(num_windows, window, qkv, order, win, scale, qkv_amax, qkv_tag, w_split, w_inv,   \
                                bias, x1, ldx1, x2, ldx2, st)                                                       \
            : launch<DD, CC, 4>(num_windows, window, qkv, order, win, scale, qkv_amax, qkv_tag, w_split, w_inv,   \
                                bias, x1, ldx1, x2, ldx2, st))
  switch (channels) {
    case 64: SFX_AP(32, 64); break;
    case 96: SFX_AP(24, 96); break;
    case 128: SFX_AP(16, 128); break;
    default: SFX_AP(16, 256); break;
  }
#undef SFX_AP
  return sfx::check_launch("sfx_window_attention_proj");
}

}  // extern "C"
