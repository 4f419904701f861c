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

// LDS-DMA piece: 16 B per lane from its own global address to M0 + 16 lane (inline asm, as subm_fused.hip: the
// builtin makes the compiler drain vmcnt whenever an address register is reused; here every wait is ours)
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds_dst) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_dst) : "memory", "m0");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Raw staging layout of a [rows][P] array of 16-byte pieces (a head's K or V slice: rows = keys, P = D / 4 float4;
// the projection slice: rows = couts, P = D / 4 pre-split groups): piece (r, p) at slot (r >> 4) 16 P + 16 p + (r & 15).
// One DMA instruction (64 consecutive slots) then reads 16 rows x P pieces -- P * 16-byte contiguous segments per
// row -- and a fragment read (32 consecutive rows, one piece) touches consecutive 16-byte slots: conflict-free.
template <int P>
__device__ __forceinline__ int raw_slot(int r, int p) { return (r >> 4) * (16 * P) + 16 * p + (r & 15); }

template <int D, int C, int NWV>
__global__ void __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2, 2)))
attn_proj_kernel(const float* __restrict__ qkv, const int* __restrict__ order, const int* __restrict__ win, int Kwin,
                 float scale, const unsigned long long* __restrict__ qkv_amax, unsigned qkv_tag,
                 const uint4* __restrict__ wsp, const float* __restrict__ winv, const float* __restrict__ bias,
                 const float* __restrict__ x1, long long ldx1, float* __restrict__ x2, long long ldx2, int nwin) {
  constexpr int H = C / D;
  constexpr int NKS = (D + 15) / 16;  // 16-deep k-steps over a head's dd (S^T contraction and projection)
  constexpr int CH = D / 4;           // 16-byte pieces per head row slice (fp32 q / k / v, pre-split Wp groups)
  constexpr int VST = 136;            // V^T row stride (16-bit elements)
  constexpr int VB = 2 * D * VST * 2;
  constexpr int KRAW = KMAX * CH * 16, WRAW = C * CH * 16;
  constexpr int RAW = 2 * KRAW + WRAW;  // one head's raw K, V and Wp slices
  constexpr int NBUF = 2 * RAW + VB <= 79 * 1024 ? 2 : 1;  // (two workgroups per CU)
  constexpr int NCB = C / 32;
  constexpr int NT = NWV * 64;
  constexpr int QPW = NWV * 32;
  constexpr int QS = KMAX / QPW;
  constexpr int KPIECES = KMAX * CH / 64, WPIECES = C * CH / 64;  // DMA instructions per slice
  static_assert(C % 32 == 0 && C % D == 0 && (KMAX * CH) % 64 == 0 && (C * CH) % 64 == 0, "shape");

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

  __shared__ __attribute__((aligned(16))) char lds[NBUF * RAW + VB];
  __shared__ int rows[KMAX];
  unsigned short* Vt = reinterpret_cast<unsigned short*>(lds + NBUF * RAW);
  const unsigned lds_base = (unsigned)(uintptr_t)lds;

  const int nb = (int)gridDim.x;
  const int L = (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8);
  if (L >= nwin * QS) return;
  const int w = L / QS, qh = L - w * QS;
  const int key_start = win[2 * w], query_start = win[2 * w + 1];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // (scalar: the DMA destinations go to M0)
  const long long ld = 3ll * C;

  // padding keys (Kwin < 128) read row 0's slices: finite values whose probability is exactly 0
  for (int r = tid; r < KMAX; r += NT) rows[r] = r < Kwin ? order[key_start + r] : -1;
  __syncthreads();

  // ---- head hd's raw K / V / Wp slices -> raw buffer `buf` by LDS-DMA (no registers held) ----
  auto issue = [&](int hd, int buf) {
    const unsigned base = lds_base + (unsigned)(buf * RAW);
#pragma unroll
    for (int i = wid; i < 2 * KPIECES; i += NWV) {  // K then V: slot i * 64 + lane of the [128][CH] piece array
      const int kv = i >= KPIECES, ii = kv ? i - KPIECES : i;
      const int sl = ii * 64 + lane;
      const int blk = sl / (16 * CH), rem = sl - blk * 16 * CH;
      const int p = rem >> 4, r = blk * 16 + (rem & 15);
      const int src = max(rows[r], 0);
      dma16(qkv + (long long)src * ld + (kv ? 2 * C : C) + hd * D + 4 * p,
            __builtin_amdgcn_readfirstlane(base + (unsigned)(kv * KRAW + ii * 1024)));
    }
#pragma unroll
    for (int i = wid; i < WPIECES; i += NWV) {  // Wp_h: [C couts][CH groups] of the pre-split
      const int sl = i * 64 + lane;
      const int blk = sl / (16 * CH), rem = sl - blk * 16 * CH;
      const int p = rem >> 4, n = blk * 16 + (rem & 15);
      dma16(wsp + (long long)n * (C / 4) + hd * CH + p,
            __builtin_amdgcn_readfirstlane(base + (unsigned)(2 * KRAW + i * 1024)));
    }
  };
  // ---- this lane's query slice of head hd (B operand of S^T = K Q^T): dd = 16 ks + 8 h + j, zero past D ----
  const int qi = QPW * qh + 32 * wid + l32;
  const int qrow = rows[qi];
  const float qs = scale * 1.4426950408889634f;  // scale * log2(e): the exponentials are plain exp2
  float4 qa[NKS], qb[NKS];
  auto load_q = [&](int hd) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int d0 = 16 * ks + 8 * h;
      qa[ks] = make_float4(0.f, 0.f, 0.f, 0.f);
      qb[ks] = qa[ks];
      if (qrow >= 0 && d0 < D) {
        const float* qp = qkv + (long long)qrow * ld + hd * D + d0;
        qa[ks] = *reinterpret_cast<const float4*>(qp);
        if (d0 + 4 < D) qb[ks] = *reinterpret_cast<const float4*>(qp + 4);
      }
    }
  };

  floatx16 y[NCB];
#pragma unroll
  for (int b = 0; b < NCB; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) y[b][r] = 0.f;

  issue(0, 0);
  load_q(0);
  wait_vm0();
  __syncthreads();

#pragma unroll 1
  for (int hd = 0; hd < H; ++hd) {
    const int buf = NBUF == 2 ? (hd & 1) : 0;
    const char* raw = lds + buf * RAW;
    // q fragments of this head (loaded one head ahead)
    f16x8 qf[NKS][2];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      float4 a = qa[ks], b = qb[ks];
      a.x *= qs; a.y *= qs; a.z *= qs; a.w *= qs;
      b.x *= qs; b.y *= qs; b.z *= qs; b.w *= qs;
      uint2 ta[2], tb[2];
      sfx::split2h(a, sq, ta);  // (|q * qs| <= |q|: the qkv bound holds)
      sfx::split2h(b, sq, tb);
#pragma unroll
      for (int q = 0; q < 2; ++q) qf[ks][q] = __builtin_bit_cast(f16x8, (uintx4){ta[q].x, ta[q].y, tb[q].x, tb[q].y});
    }
    if (NBUF == 2 && hd + 1 < H) {  // the next head's slices fly while this one computes
      issue(hd + 1, buf ^ 1);
      load_q(hd + 1);
    }
    // V^T image of this head from the raw V slice (key pairs x float4: whole-dword transposed stores)
    for (int e = tid; e < (KMAX / 2) * CH; e += NT) {
      const int kp = e / CH, ch = e - kp * CH;
      const int row = 2 * kp;
      const float4 v0 = *reinterpret_cast<const float4*>(raw + KRAW + 16 * raw_slot<CH>(row, ch));
      const float4 v1 = *reinterpret_cast<const float4*>(raw + KRAW + 16 * raw_slot<CH>(row + 1, ch));
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
    __syncthreads();  // V^T written

    // ---- S^T[key][query] -> softmax -> O^T[dd][query] = V^T P^T, in NPASS passes over the 128 keys (online
    // softmax across passes: C = 256's 128 projection accumulators leave room for 64 score registers, not 128) ----
    constexpr int NPASS = NCB >= 8 ? 2 : 1, KBP = 4 / NPASS;
    const float iqq = iq * iq;
    float mx = -INFINITY, sum = 0.f;
    floatx16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      floatx16 s[KBP];
#pragma unroll
      for (int j = 0; j < KBP; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[j][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int j = 0; j < KBP; ++j) {  // K fragments split from the raw slice as they are read
          const int kb = ps * KBP + j, p0 = 4 * ks + 2 * h;
          float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
          if (4 * p0 < D) {
            a = *reinterpret_cast<const float4*>(raw + 16 * raw_slot<CH>(kb * 32 + l32, p0));
            b = *reinterpret_cast<const float4*>(raw + 16 * raw_slot<CH>(kb * 32 + l32, p0 + 1));
          }
          uint2 ta[2], tb[2];
          sfx::split2h(a, sq, ta);
          sfx::split2h(b, sq, tb);
          const f16x8 kh = __builtin_bit_cast(f16x8, (uintx4){ta[0].x, ta[0].y, tb[0].x, tb[0].y});
          const f16x8 kl = __builtin_bit_cast(f16x8, (uintx4){ta[1].x, ta[1].y, tb[1].x, tb[1].y});
          s[j] = mfma16(kl, qf[ks][0], s[j]);
          s[j] = mfma16(kh, qf[ks][1], s[j]);
          s[j] = mfma16(kh, qf[ks][0], s[j]);
        }
      float pm = -INFINITY;
#pragma unroll
      for (int j = 0; j < KBP; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = s[j][r] * iqq;
          const int key = (ps * KBP + j) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (Kwin < KMAX && key >= Kwin) v = -INFINITY;
          s[j][r] = v;
          pm = fmaxf(pm, v);
        }
      pm = fmaxf(pm, __shfl_xor(pm, 32, 64));
      const float mn = fmaxf(mx, pm);  // finite: every window has >= 1 key in pass 0
      if (ps > 0) {
        const float al = __builtin_amdgcn_exp2f(mx - mn);
        sum *= al;
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] *= al;
      }
      mx = mn;
      float ps_sum = 0.f;
#pragma unroll
      for (int j = 0; j < KBP; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float ex = __builtin_amdgcn_exp2f(s[j][r] - mx);
          s[j][r] = ex;
          ps_sum += ex;
        }
      sum += ps_sum + __shfl_xor(ps_sum, 32, 64);
#pragma unroll
      for (int j = 0; j < KBP; ++j)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int kb = ps * KBP + j;
          uint2 a[2], b[2];
          sfx::split2h(make_float4(s[j][8 * st + 0], s[j][8 * st + 1], s[j][8 * st + 2], s[j][8 * st + 3]), 16384.f, a);
          sfx::split2h(make_float4(s[j][8 * st + 4], s[j][8 * st + 5], s[j][8 * st + 6], s[j][8 * st + 7]), 16384.f, b);
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
    }
    const float rinv = 1.f / sum;

    // ---- Y^T[cout][query] += Wp_h O_h^T: O^T (x sq) as fp16 terms from registers 8s..8s+7 (k-step s, permuted
    // order dd = 16 s + 8 (j >> 2) + 4 h + (j & 3): groups 4 s + h and 4 s + 2 + h of the pre-split Wp rows) ----
    const float osc = rinv * (1.f / 16384.f);  // o = 2^14 sq sum_k p v  ->  O sq
#pragma unroll
    for (int sp = 0; sp < NKS; ++sp) {
      uint2 a[2], b[2];
      sfx::split2h(make_float4(o[8 * sp + 0], o[8 * sp + 1], o[8 * sp + 2], o[8 * sp + 3]), osc, a);
      sfx::split2h(make_float4(o[8 * sp + 4], o[8 * sp + 5], o[8 * sp + 6], o[8 * sp + 7]), osc, b);
      const f16x8 oh = __builtin_bit_cast(f16x8, make_uint4(a[0].x, a[0].y, b[0].x, b[0].y));
      const f16x8 ol = __builtin_bit_cast(f16x8, make_uint4(a[1].x, a[1].y, b[1].x, b[1].y));
      const int g0 = 4 * sp + h, g1 = g0 + 2;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        uint4 wa = make_uint4(0, 0, 0, 0), wb = wa;
        if (4 * g0 < D) wa = *reinterpret_cast<const uint4*>(raw + 2 * KRAW + 16 * raw_slot<CH>(cb * 32 + l32, g0));
        if (4 * g1 < D) wb = *reinterpret_cast<const uint4*>(raw + 2 * KRAW + 16 * raw_slot<CH>(cb * 32 + l32, g1));
        const f16x8 wh = __builtin_bit_cast(f16x8, make_uint4(wa.x, wa.y, wb.x, wb.y));
        const f16x8 wl = __builtin_bit_cast(f16x8, make_uint4(wa.z, wa.w, wb.z, wb.w));
        y[cb] = mfma16(wl, oh, y[cb]);
        y[cb] = mfma16(wh, ol, y[cb]);
        y[cb] = mfma16(wh, oh, y[cb]);
      }
    }
    if (hd + 1 < H) {
      if (NBUF == 1) {  // single raw buffer: fetch the next head only after every wave is done with this one
        __syncthreads();
        issue(hd + 1, 0);
        load_q(hd + 1);
      }
      wait_vm0();       // this thread's DMAs (and q loads) of the next head have landed
      __syncthreads();  // ... and everyone's: the next head's raw slices are visible, this head's reads are done
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
  (void)nwin;
  return 4;  // (the raw double buffer is per workgroup: half-window workgroups would stage every slice twice)
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
