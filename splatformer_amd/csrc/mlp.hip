// Fused PTv3 Block MLP tail (eval): Y = X2 + fc2(GELU(fc1(LN2(X2))))  -- reference Block.forward, restated in
// calflops.py:72-82 (norm2 -> mlp -> drop_path(identity in eval) -> + shortcut), MLP = Linear(C,4C) -> GELU
// (erf) -> Linear(4C,C) (pointtransformer_v3.py:145, Pointcept MLP).
//
// One launch replaces LayerNorm + two GEMMs: the [M, C] LayerNorm output and the [M, 4C] hidden activation never
// reach HBM (in the unfused form they are written and read back: 10 C floats per point, 8.6 GB per config-B
// refine).  HBM traffic is the algorithmic X2 read + Y write; the weights stream from L2.
//
// Arithmetic: fp32-accurate fp16x2 MFMA (the GEMM family's scheme, gemm.hip): every operand is a power-of-two
// scaled pair of fp16 terms h + l and every 32x32x16 block is h*h + h*l + l*h on v_mfma_f32_32x32x16_f16 with
// fp32 accumulation.  Scales:
//   * LN2 output row p: its exact row maximum (known here: the whole row is LayerNormed in the workgroup) in
//     [2^13, 2^14);
//   * hidden row p (all 4C units, every chunk): one scale from the bound |GELU(z)| <= max(|z|, 0.17),
//     |z_u| <= ||LN2(x)_p||_2 max_u ||W1_u||_2 + max|b1| (Cauchy-Schwarz; the bound puts the row in [2^14, 2^15)
//     at most, so no chunk overflows fp16 and no running rescale is needed);
//   * W1 rows / W2 rows: their own maxima in [2^14, 2^15) (pre-split once per weight version, sfx_mlp_pack).
//
// Work decomposition (mlp_kernel below): one workgroup = WAVES x 32 points, wave w owns 32 points and computes
// every hidden unit and every output channel for them.  The hidden layer is processed in chunks of 64 units.
// Computed transposed (points on the lanes): per chunk, the wave forms hid^T[2 x 32 units, 32 points] =
// W1_chunk . LN2(X2)^T (A = W1 rows from the LDS ring, B = the wave's LN2 fragments held in registers), applies
// bias + GELU + split in registers, and feeds the accumulator registers straight back as the B operand of fc2 (a
// 32x32 accumulator's registers 8s..8s+7 are the k-step s fragment of A.X, the k order permuted:
// cdna_hip_programming.md §3) -- the hidden never touches LDS either.  fc2^T: acc2^T[C channels, 32 points] +=
// W2[:, the chunk's 64 units] . hid^T, kept in registers for the whole tile.
//
// Weights stream through an LDS ring by LDS-DMA (global_load_lds_dwordx4): sfx_mlp_pack lays W1 / W2 out as
// 8 KB slabs in exactly the swizzled order the fragments are read in (so a slab is a plain contiguous copy) and in
// consumption order: per chunk C/32 fc1 slabs ([2 halves][2 terms][32 units][32 k]) then C/32 fc2 slabs
// ([2 halves][2 terms][32 channels][32 units, permuted]).  A phase = 2 slabs (16 KB) = 12 MFMAs per wave; the ring
// holds RING phases, RING-1 in flight; one barrier per phase (RAW for the arriving slabs, WAR for the refilled
// slot), counted vmcnt, raw s_barrier (no __syncthreads: its fence would drain the DMA queue).
#include <map>
#include <mutex>
#include <cstdlib>

#include "gemm_common.h"

extern "C" int sfx_get_precision(void);  // gemm.hip (include/sfx.h)

#ifndef SFX_MLP_RING256
#define SFX_MLP_RING256 8  // LDS ring phases of the C = 256 kernel
#endif

namespace {

using namespace sfxg;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int SLAB_BYTES = 8192;    // one streamed weight slab
constexpr int PHASE_BYTES = 2 * SLAB_BYTES;

template <int C>
struct MlpGeom {
  static constexpr int NB = C / 32;           // 32-channel blocks = fc1 slabs per chunk = fc2 slabs per chunk
  static constexpr int NCH = C / 16;          // hidden chunks of 64 units (4C / 64)
  static constexpr int PPC = NB;              // phases per chunk (2 * NB slabs, 2 per phase)
  static constexpr int NP = NCH * PPC;        // phases per tile
  static constexpr int PAR = 12 * C + 4;      // parameter table floats
};

// Parameter table (floats): [0,C) gamma, [C,2C) beta, [2C,10C) (1/s_u, b1_u) pairs in fc1-epilogue order,
// [10C,12C) (1/s_c, b2_c) pairs in fc2-epilogue order, [12C] max_u ||W1_u||_2, [12C+1] max |b1|.
__device__ __forceinline__ int fc1_par_index(int j, int cn, int h, int i) { return ((j * 2 + cn) * 2 + h) * 16 + i; }
__device__ __forceinline__ int fc2_par_index(int b, int h, int i) { return (b * 2 + h) * 16 + i; }
// accumulator register i of lane half h -> row within the 32-row block (MFMA 32x32 C/D layout)
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
// byte offset of fp16 element q (0..31) of row r in a swizzled [32 rows][64 B] term image (16-B chunk c at
// c ^ ((r >> 2) & 3): the fragment reads of 16 rows x one chunk are bank-conflict free)
__device__ __forceinline__ int slab_off(int r, int q) {
  return r * 64 + ((((q >> 3) ^ (r >> 2)) & 3) << 4) + ((q & 7) << 1);
}

// Before each phase's barrier: (RAW) this wave's DMAs of the phase about to be read have landed -- the younger
// phases in flight (PIECES each) may still fly; (WAR) its LDS reads of the previous phase have returned
// (lgkmcnt(0)), so the slot the phase refills after the barrier is no longer being read (cdna_hip_programming.md
// §5, "Read a staged buffer one phase AFTER the wait that retires it": a slot restaged one phase after its last
// read needs that lgkmcnt before the barrier).
template <int N>
__device__ __forceinline__ void wait_vm_lgkm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

// One workgroup = WAVES x 32 points; wave w owns points [32 w, 32 w + 32) of the tile and computes every hidden
// unit and every output channel for them, so nothing but the weights is shared: the LN2 output of a wave's points
// lives in its registers as the fc1 B fragments (lane (r, h) holds point r's channels 16 t + 8 h .. + 7 for every
// k-step t -- half a row per lane, LayerNorm statistics completed with the partner lane r + 32), and the weights
// are read from the LDS ring by all WAVES waves (WAVES-fold reuse per DMA'd byte).
// HS (hidden split): a PAIR of waves owns 32 points, wave cn = wid & 1 taking the 32-unit half cn of every 64-unit
// hidden chunk (half the fc1 / GELU / fc2 work and LDS reads per wave); the two partial fc2 sums meet once through
// LDS at the end (cn 0 + cn 1, a fixed order).  Twice the waves per point: at C = 256 (37759 points, one 512-register
// wave per SIMD) 1180 whole-tile waves over 1024 SIMDs take two full rounds, 2360 half-work waves take three half
// rounds.
// KIND (training, configs C/D -- the same dataflow, other operands):
//   MLP_EVAL  Y = X + fc2(GELU(fc1(LN2(X))));
//   MLP_TRAIN the training forward: also stores the pre-activation Z = fc1(LN2(X)) [M, 4C] for the backward, and
//             scales the branch by the DropPath keep mask: Y = X + rs[p] (fc2(GELU(Z)) + b2);
//   MLP_BWD   the branch's input gradient before LN2's backward: Y = W1^T (GELU'(Z) o (W2^T (rs[p] dY))) -- packed
//             with W2^T in fc1's place and W1^T in fc2's (zero biases, sfx_block_mlp_bwd_pack), X = dY, no
//             LayerNorm, Z read back instead of stored; hidden bound ||rs dY|| max_u ||W2[:, u]|| max|GELU'|.
enum MlpKind { MLP_EVAL = 0, MLP_TRAIN = 1, MLP_BWD = 2 };

// GELU'(z) = Phi(z) + z phi(z) with gelu_erf's fitted Phi (one exp2 for the tail, one for the density): ~20 VALU,
// branch-free, against erff + expf (gelu_erf_grad) whose branches and temporaries spill the C = 96 backward tile
__device__ __forceinline__ float gelu_grad_fit(float x) {
  const float t = fminf(fabsf(x), 5.65f);
  float q = 2.79405867e-06f;
  q = __builtin_fmaf(q, t, -3.89084234e-05f);
  q = __builtin_fmaf(q, t, 0.000184072458f);
  q = __builtin_fmaf(q, t, 0.000141672252f);
  q = __builtin_fmaf(q, t, -0.00706906663f);
  q = __builtin_fmaf(q, t, 0.0524996631f);
  q = __builtin_fmaf(q, t, 0.459207207f);
  q = __builtin_fmaf(q, t, 1.15110528f);
  const float half_tail = 0.5f * __builtin_amdgcn_exp2f(-(t * q));
  const float phi_cdf = x >= 0.f ? 1.f - half_tail : half_tail;
  return phi_cdf + x * (0.39894228040143268f * __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x));
}

// ONE (training kinds under sfx_set_precision(1), the reference's autocast class): the leading product h*h of each
// block only (the l terms are never read: fp16-rounded operands, fp32 accumulation).
// SPLIT > 1 (eval; the last, partial round of a launch -- sfx_block_mlp's tail): workgroup (x, s) computes the
// hidden chunks [s NCH / SPLIT, (s + 1) NCH / SPLIT) of its points only and stores its fc2 partial sum (+ b2 for
// s = 0) as row x of P [SPLIT][M][C]; mlp_combine_kernel adds X and the SPLIT partials in a fixed order.  The tail
// then takes 1 / SPLIT of a round instead of a whole one.
template <int C, int WAVES, int RING, bool HS = false, int KIND = MLP_EVAL, bool ONE = false, int SPLIT = 1>
__global__ void __launch_bounds__(WAVES * 64, (WAVES == 4 && C > 128) ? 1 : 2)
    mlp_kernel(int M, const float* __restrict__ X, long long ldx, const float* __restrict__ stream,
               const float* __restrict__ par, float eps, float* __restrict__ Y, long long ldy, int rot,
               const float* __restrict__ rowscale, float* __restrict__ Z, float* __restrict__ P = nullptr) {
  using G = MlpGeom<C>;
  constexpr int PTS = HS ? WAVES * 16 : WAVES * 32;  // points per workgroup
  static_assert(G::NCH % SPLIT == 0, "hidden-chunk split: whole chunks");
  constexpr int NCHS = G::NCH / SPLIT;                // hidden chunks of this workgroup
  constexpr int NB = G::NB, NP = NCHS * G::PPC, PPC = G::PPC, NT = C / 16;  // NT: fc1 k-steps
  constexpr int NTH = WAVES * 64;
  constexpr int PIECES = 16 / WAVES;  // 1 KB LDS-DMA pieces per wave per phase
  constexpr int PAR_OFF = RING * PHASE_BYTES;
  constexpr int LDS_BYTES = PAR_OFF + G::PAR * 4;
  static_assert(16 % WAVES == 0 && LDS_BYTES <= 163840, "geometry");
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float* s_par = reinterpret_cast<float*>(lds + PAR_OFF);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int cn = HS ? (wid & 1) : 0;        // HS: this wave's hidden half
  const int pg = HS ? (wid >> 1) : wid;      // this wave's 32-point group
  const int prow = (int)blockIdx.x * PTS + pg * 32 + r32;  // this lane's point
  const bool pok = prow < M;

  // ---- weight stream: logical phase q -> ring slot q % RING; rot: each workgroup starts at its own hidden
  // chunk j0 and wraps, so the workgroups of an XCD read different parts of the stream at any moment
  const int j0 = SPLIT > 1 ? (int)blockIdx.y * NCHS : (rot ? (int)(blockIdx.x % G::NCH) : 0);
  const char* gstream = reinterpret_cast<const char*>(stream);
  auto issue = [&](int q) {
    int jq = q / PPC + j0;
    jq -= jq >= G::NCH ? G::NCH : 0;
    const int sq = jq * PPC + (q - (q / PPC) * PPC);  // stream phase of logical phase q
    const char* src = gstream + (size_t)sq * PHASE_BYTES + wid * (PIECES * 1024) + lane * 16;
    char* dst = lds + (q % RING) * PHASE_BYTES + wid * (PIECES * 1024);
#pragma unroll
    for (int pc = 0; pc < PIECES; ++pc)
      __builtin_amdgcn_global_load_lds(src + pc * 1024, (__attribute__((address_space(3))) void*)(dst + pc * 1024),
                                       16, 0, 0);
  };
#pragma unroll
  for (int q = 0; q < RING - 1; ++q)
    if (q < NP) issue(q);

  // ---- prologue: parameter table; this lane's half row of X2, LayerNorm, fc1 B fragments, scales ----
  for (int i = tid; i < G::PAR; i += NTH) s_par[i] = par[i];
  const __amdgpu_buffer_rsrc_t rX = rsrc_ext(X, (unsigned)M * (unsigned)ldx * 4u);
  const unsigned xr = (unsigned)prow * (unsigned)ldx;
  float4 v[2 * NT];  // channels 16 t + 8 h + 0..3 (v[2t]) and + 4..7 (v[2t+1])
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const unsigned c = (unsigned)(16 * t + 8 * h);
    v[2 * t] = bload4(rX, pok ? (xr + c) * 4u : OOB);
    v[2 * t + 1] = bload4(rX, pok ? (xr + c + 4u) * 4u : OOB);
  }
  // the DropPath keep factor of this point (training kinds; 1 without a mask, 0 past M)
  const float rsp = (KIND != MLP_EVAL && rowscale) ? (pok ? rowscale[prow] : 0.f) : 1.f;
  float mean = 0.f, rstd = 1.f;
  if constexpr (KIND != MLP_BWD) {
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i) sm += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    sm += __shfl_xor(sm, 32, 64);
    mean = sm / (float)C;
    float q2 = 0.f;
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i) {
      const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
      q2 += (a * a + b * b) + (c * c + d * d);
    }
    q2 += __shfl_xor(q2, 32, 64);
    rstd = 1.f / sqrtf(q2 / (float)C + eps);
  }
  __syncthreads();  // s_par visible (no DMA is waited for here: only plain stores precede it)
  float mx = 0.f, nrm = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = 16 * t + 8 * h + 4 * u;
      float4& w = v[2 * t + u];
      if constexpr (KIND != MLP_BWD) {
        const float4 g = *reinterpret_cast<const float4*>(s_par + c);
        const float4 b = *reinterpret_cast<const float4*>(s_par + C + c);
        w = make_float4((w.x - mean) * rstd * g.x + b.x, (w.y - mean) * rstd * g.y + b.y,
                        (w.z - mean) * rstd * g.z + b.z, (w.w - mean) * rstd * g.w + b.w);
      } else {  // dY of the branch output = rs[p] * dY
        w = make_float4(w.x * rsp, w.y * rsp, w.z * rsp, w.w * rsp);
      }
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(w.x), fabsf(w.y)), fmaxf(fabsf(w.z), fabsf(w.w))));
      nrm += (w.x * w.x + w.y * w.y) + (w.z * w.z + w.w * w.w);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  nrm += __shfl_xor(nrm, 32, 64);
  int e = 0;
  if (mx > 0.f && mx <= 3.4028235e38f) e = row_exp(mx) + 1;  // row max in [2^13, 2^14)
  const float sc = ldexpf(1.f, e), sinv = ldexpf(1.f, -e);
  // hidden bound: |GELU(z)| <= max(|z|, 0.17), |z| <= ||h2|| max||W1_u|| + max|b1| (1.001: the sums' rounding);
  // backward: |GELU'(z) (W2^T dy)_u| <= 1.13 ||dy|| max_u ||W2[:, u]|| (max GELU' = 1.129 at z = sqrt 2)
  const float U = KIND == MLP_BWD ? fmaxf(sqrtf(nrm) * s_par[12 * C] * (1.13f * 1.001f), 1e-30f)
                                  : fmaxf((sqrtf(nrm) * s_par[12 * C] + s_par[12 * C + 1]) * 1.001f, 0.17f);
  int et = 0;
  if (U <= 3.4028235e38f) et = row_exp(U) + 2;  // bound in [2^14, 2^15)
  const float tsc = ldexpf(1.f, et), tinv = ldexpf(1.f, -et);
  f16x8 hb[NT][2];  // fc1 B fragments [k-step][term]
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    uint2 lo[2], hi[2];
    split2h(v[2 * t], sc, lo);
    split2h(v[2 * t + 1], sc, hi);
    hb[t][0] = __builtin_bit_cast(f16x8, make_uint4(lo[0].x, lo[0].y, hi[0].x, hi[0].y));
    hb[t][1] = __builtin_bit_cast(f16x8, make_uint4(lo[1].x, lo[1].y, hi[1].x, hi[1].y));
  }

  floatx16 acc2[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc2[b][i] = 0.f;
  floatx16 acc1[2];
  f16x8 hf[2][2][2];  // hidden fragments: [unit block][k-step][term]

  auto mfma3 = [](const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, floatx16 c) {
    if constexpr (ONE) return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);  // smallest terms first
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  };

  // the 8 fragment pairs of one slab (both 32-row halves x 2 k-steps x 2 terms), read in one batch so the LDS
  // latency is paid once per slab, not once per MFMA triple
  auto load_frags = [&](const char* base, f16x8 (&fa)[2][2][2]) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (HS && cb != 0) break;              // HS: the own half only, in slot 0
        const char* half = base + (HS ? cn : cb) * 4096;
        const int o = slab_off(r32, 16 * t + 8 * h);
        fa[cb][t][0] = *reinterpret_cast<const f16x8*>(half + o);
        fa[cb][t][1] = *reinterpret_cast<const f16x8*>(half + 2048 + o);
      }
  };
  // one slab: sl < NB -> fc1 slab sl (input channels 32 sl .. +32, both 32-unit blocks), else fc2 slab sl - NB
  auto slab = [&](const f16x8 (&fa)[2][2][2], int sl, int j) {
    constexpr int NCB = HS ? 1 : 2;  // unit blocks of a chunk this wave computes
    if (sl < NB) {
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc1[cb] = mfma3(fa[cb][t][0], fa[cb][t][1], hb[2 * sl + t][0], hb[2 * sl + t][1], acc1[cb]);
      if (sl == NB - 1) {  // hidden chunk complete: bias, GELU, split -> fc2 B fragments (registers)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const float4* pp =
              reinterpret_cast<const float4*>(s_par + 2 * C + 2 * fc1_par_index(j, HS ? cn : cb, h, 0));
          float g[16];
          // Z row of this lane's point: registers 4 q .. 4 q + 3 are units 64 j + 32 cb' + 8 q + 4 h + 0..3
          float* zrow = Z + (size_t)(pok ? prow : 0) * (4 * C) + 64 * j + 32 * (HS ? cn : cb) + 4 * h;
          if constexpr (KIND == MLP_BWD) {
            float4 zq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
              zq[q] = pok ? *reinterpret_cast<const float4*>(zrow + 8 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int i2 = 0; i2 < 8; ++i2) {
              const float4 wb = pp[i2];  // (1/s_u, 0) of registers 2 i2, 2 i2 + 1
              const float4 zz = zq[i2 >> 1];
              g[2 * i2 + 0] = acc1[cb][2 * i2 + 0] * (sinv * wb.x) * gelu_grad_fit((i2 & 1) ? zz.z : zz.x) * tsc;
              g[2 * i2 + 1] = acc1[cb][2 * i2 + 1] * (sinv * wb.z) * gelu_grad_fit((i2 & 1) ? zz.w : zz.y) * tsc;
            }
          } else {
            float pre[16];
#pragma unroll
            for (int i2 = 0; i2 < 8; ++i2) {
              const float4 wb = pp[i2];  // (1/s_u, b1_u) of registers 2 i2, 2 i2 + 1
              pre[2 * i2 + 0] = acc1[cb][2 * i2 + 0] * (sinv * wb.x) + wb.y;
              pre[2 * i2 + 1] = acc1[cb][2 * i2 + 1] * (sinv * wb.z) + wb.w;
            }
            if constexpr (KIND == MLP_TRAIN) {
              if (pok)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  *reinterpret_cast<float4*>(zrow + 8 * q) =
                      make_float4(pre[4 * q], pre[4 * q + 1], pre[4 * q + 2], pre[4 * q + 3]);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) g[i] = gelu_erf(pre[i]) * tsc;
          }
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            unsigned uh[4], ul[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float x0 = g[8 * st + 2 * k], x1 = g[8 * st + 2 * k + 1];
              uh[k] = sfx::pk_f16(x0, x1);
              const sfx::sfx_f16x2 hh = __builtin_bit_cast(sfx::sfx_f16x2, uh[k]);
              ul[k] = sfx::pk_f16(x0 - (float)hh.x, x1 - (float)hh.y);
            }
            hf[cb][st][0] = __builtin_bit_cast(f16x8, make_uint4(uh[0], uh[1], uh[2], uh[3]));
            hf[cb][st][1] = __builtin_bit_cast(f16x8, make_uint4(ul[0], ul[1], ul[2], ul[3]));
          }
        }
      }
    } else {
      const int b = sl - NB;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int st = 0; st < 2; ++st)
          acc2[b] = mfma3(fa[cb][st][0], fa[cb][st][1], hf[cb][st][0], hf[cb][st][1], acc2[b]);
    }
  };

  int p = 0;
  for (int jl = 0; jl < NCHS; ++jl) {
    const int j = jl + j0 - (jl + j0 >= G::NCH ? G::NCH : 0);  // the hidden chunk of this logical chunk
#pragma unroll
    for (int cb = 0; cb < (HS ? 1 : 2); ++cb)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc1[cb][i] = 0.f;
#pragma unroll
    for (int pi = 0; pi < PPC; ++pi, ++p) {
      if (p + RING - 1 < NP) wait_vm_lgkm<(RING - 2) * PIECES>();
      else wait_vm_lgkm<0>();  // tail: nothing younger than this phase in flight
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");  // no LDS access moves across the barrier
      if (p + RING - 1 < NP) issue(p + RING - 1);  // refills the slot every wave finished before the barrier
      const char* base = lds + (p % RING) * PHASE_BYTES;
      f16x8 fa0[2][2][2], fa1[2][2][2];
      load_frags(base, fa0);
      load_frags(base + SLAB_BYTES, fa1);
      slab(fa0, 2 * pi, j);
      slab(fa1, 2 * pi + 1, j);
    }
  }

  if constexpr (HS) {  // the cn = 1 wave's partial fc2 sums -> LDS (the drained ring) -> added by its cn = 0 partner
    static_assert((WAVES / 2) * 64 * NB * 16 * 4 <= RING * PHASE_BYTES, "HS exchange fits the ring");
    __builtin_amdgcn_s_barrier();  // every wave's last ring reads are done (the tail waited for every DMA)
    asm volatile("" ::: "memory");
    float4* xch = reinterpret_cast<float4*>(lds) + (size_t)pg * 64 * NB * 4;
    if (cn == 1) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          xch[(b * 4 + q) * 64 + lane] = make_float4(acc2[b][4 * q], acc2[b][4 * q + 1], acc2[b][4 * q + 2],
                                                     acc2[b][4 * q + 3]);
    }
    __syncthreads();
    if (cn == 1) return;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 o = xch[(b * 4 + q) * 64 + lane];
        acc2[b][4 * q] += o.x;
        acc2[b][4 * q + 1] += o.y;
        acc2[b][4 * q + 2] += o.z;
        acc2[b][4 * q + 3] += o.w;
      }
  }
  // ---- epilogue: Y = X2 + acc2 / (t s_c) + b2, 16-byte stores of 4 consecutive channels ----
  const __amdgpu_buffer_rsrc_t rY = rsrc_ext(Y, (unsigned)M * (unsigned)ldy * 4u);
  const unsigned yr = (unsigned)prow * (unsigned)ldy;
  float ymax = 0.f;  // MLP_EVAL with Z: this point's max |Y| -> the next fused SubM conv's row exponent
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const float4* pp = reinterpret_cast<const float4*>(s_par + 10 * C + 2 * fc2_par_index(b, h, 0));
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float4 w01 = pp[2 * g4], w23 = pp[2 * g4 + 1];  // (1/s_c, b2_c) of registers 4 g4 .. 4 g4 + 3
      const unsigned c0 = (unsigned)(32 * b + 8 * g4 + 4 * h);
      float4 y;
      if constexpr (SPLIT > 1) {  // this split's branch partial (b2 carried by split 0) -> P[s][prow]
        const float bb = (KIND != MLP_BWD && blockIdx.y == 0) ? 1.f : 0.f;
        const float rr = KIND == MLP_BWD ? 1.f : rsp;  // (BWD: rs is applied to dY in the prologue)
        y.x = rr * (acc2[b][4 * g4 + 0] * (tinv * w01.x) + bb * w01.y);
        y.y = rr * (acc2[b][4 * g4 + 1] * (tinv * w01.z) + bb * w01.w);
        y.z = rr * (acc2[b][4 * g4 + 2] * (tinv * w23.x) + bb * w23.y);
        y.w = rr * (acc2[b][4 * g4 + 3] * (tinv * w23.z) + bb * w23.w);
        if (pok)
          *reinterpret_cast<float4*>(P + ((size_t)blockIdx.y * M + prow) * C + c0) = y;
        continue;
      } else if constexpr (KIND == MLP_BWD) {  // the branch's input gradient: no bias, no residual
        y.x = acc2[b][4 * g4 + 0] * (tinv * w01.x);
        y.y = acc2[b][4 * g4 + 1] * (tinv * w01.z);
        y.z = acc2[b][4 * g4 + 2] * (tinv * w23.x);
        y.w = acc2[b][4 * g4 + 3] * (tinv * w23.z);
      } else {
        const float4 xres = bload4(rX, pok ? (xr + c0) * 4u : OOB);
        y.x = xres.x + rsp * (acc2[b][4 * g4 + 0] * (tinv * w01.x) + w01.y);
        y.y = xres.y + rsp * (acc2[b][4 * g4 + 1] * (tinv * w01.z) + w01.w);
        y.z = xres.z + rsp * (acc2[b][4 * g4 + 2] * (tinv * w23.x) + w23.y);
        y.w = xres.w + rsp * (acc2[b][4 * g4 + 3] * (tinv * w23.z) + w23.w);
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), rY, pok ? (yr + c0) * 4u : OOB, 0, 0);
      if constexpr (KIND == MLP_EVAL) ymax = fmaxf(ymax, fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
    }
  }
  if constexpr (KIND == MLP_EVAL && SPLIT == 1) {
    // sfx_subm_rowexp of the output row (csrc/subm_fused.hip, same rule): max in [2^14, 2^15), 127 for a zero row,
    // 0 for inf / nan -- the next Block's fused conv reads it instead of re-reading the row
    if (Z) {
      ymax = fmaxf(ymax, __shfl_xor(ymax, 32, 64));
      if (h == 0 && pok) {
        int e = 127;
        if (ymax > 0.f && ymax <= 3.4028235e38f) {
          e = 15 - __builtin_amdgcn_frexp_expf(ymax);
          e = e > 126 ? 126 : (e < -126 ? -126 : e);
        } else if (!(ymax <= 3.4028235e38f)) {
          e = 0;
        }
        reinterpret_cast<int*>(Z)[prow] = e;
      }
    }
  }
}

// Y = X + (P[0] + P[1] + ... + P[S-1]) for the rows of a split tail (fixed order: bitwise reproducible); one wave
// per row, lane i < C / 4 owns channels 4i .. 4i + 3; rowexp (optional): the MLP_EVAL epilogue's row-exponent rule
template <int S>
__global__ void __launch_bounds__(256) mlp_combine_kernel(int M, int C, const float* __restrict__ X, long long ldx,
                                                          const float* __restrict__ P, float* __restrict__ Y,
                                                          long long ldy, int* __restrict__ rowexp) {
  const int r = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= M) return;
  float m = 0.f;
  if (lane < C / 4) {
    const int c = 4 * lane;
    float4 a = *reinterpret_cast<const float4*>(P + (size_t)r * C + c);
#pragma unroll
    for (int q = 1; q < S; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(P + ((size_t)q * M + r) * C + c);
      a = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
    const float4 x = X ? *reinterpret_cast<const float4*>(X + (size_t)r * ldx + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 y = X ? make_float4(x.x + a.x, x.y + a.y, x.z + a.z, x.w + a.w) : a;
    *reinterpret_cast<float4*>(Y + (size_t)r * ldy + c) = y;
    m = fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w)));
  }
  if (rowexp) {
    m = sfx::wave_max(m);
    if (lane == 0) {
      int e = 127;
      if (m > 0.f && m <= 3.4028235e38f) {
        e = 15 - __builtin_amdgcn_frexp_expf(m);
        e = e > 126 ? 126 : (e < -126 ? -126 : e);
      } else if (!(m <= 3.4028235e38f)) {
        e = 0;
      }
      rowexp[r] = e;
    }
  }
}

// ---- weight packing (once per weight version) ----------------------------------------------------------------
// per-row exponents (max in [2^14, 2^15)) and W1 row norms
__global__ void __launch_bounds__(256) mlp_rowstats_kernel(int rows, int cols, const float* __restrict__ W,
                                                           int* __restrict__ e_out, float* __restrict__ nrm_out) {
  const int row = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float m = 0.f, s = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float x = W[(long long)row * cols + c];
    m = fmaxf(m, fabsf(x));
    s += x * x;
  }
  m = sfx::wave_max(m);
  s = sfx::wave_sum(s);
  if (lane == 0) {
    e_out[row] = (m > 0.f && m <= 3.4028235e38f) ? row_exp(m) + 2 : 0;
    if (nrm_out) nrm_out[row] = sqrtf(s);
  }
}

// one thread per (slab, half, row, position): both terms of one element
template <int C>
__global__ void __launch_bounds__(256) mlp_pack_stream_kernel(const float* __restrict__ W1,
                                                              const float* __restrict__ W2, const int* __restrict__ e1,
                                                              const int* __restrict__ e2, float* __restrict__ stream) {
  using G = MlpGeom<C>;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)G::NCH * 2 * G::NB * 2 * 32 * 32;
  if (idx >= total) return;
  const int q = (int)(idx & 31), r = (int)((idx >> 5) & 31), cn = (int)((idx >> 10) & 1);
  const long long sidx = idx >> 11;  // slab index in stream order
  const int j = (int)(sidx / (2 * G::NB)), sl = (int)(sidx % (2 * G::NB));
  float w;
  int e;
  if (sl < G::NB) {  // fc1 slab: row r = unit 64 j + 32 cn + r, position q = input channel 32 sl + q
    const int u = 64 * j + 32 * cn + r;
    w = W1[(long long)u * C + 32 * sl + q];
    e = e1[u];
  } else {  // fc2 slab: row r = channel 32 b + r, position q = k-step q >> 4, lane half / element -> unit
    const int b = sl - G::NB, c = 32 * b + r;
    const int st = q >> 4, qq = q & 15, hh = qq >> 3, jj = qq & 7;
    const int u = 64 * j + 32 * cn + 16 * st + 8 * (jj >> 2) + 4 * hh + (jj & 3);
    w = W2[(long long)c * (4 * C) + u];
    e = e2[c];
  }
  const float x = w * ldexpf(1.f, e);
  const _Float16 hv = (_Float16)x;
  const _Float16 lv = (_Float16)(x - (float)hv);
  char* slab = reinterpret_cast<char*>(stream) + sidx * SLAB_BYTES + cn * 4096;
  *reinterpret_cast<_Float16*>(slab + slab_off(r, q)) = hv;
  *reinterpret_cast<_Float16*>(slab + 2048 + slab_off(r, q)) = lv;
}

template <int C>
__global__ void __launch_bounds__(256) mlp_pack_params_kernel(const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              const float* __restrict__ b1,
                                                              const float* __restrict__ b2, const int* __restrict__ e1,
                                                              const int* __restrict__ e2, const float* __restrict__ n1,
                                                              float* __restrict__ par) {
  using G = MlpGeom<C>;
  const int tid = (int)blockIdx.x * 256 + threadIdx.x;
  if (tid < C) {
    par[tid] = gamma[tid];
    par[C + tid] = beta[tid];
  }
  if (tid < 4 * C) {  // fc1 entry tid = ((j * 2 + cn) * 2 + h) * 16 + i
    const int i = tid & 15, hh = (tid >> 4) & 1, cn = (tid >> 5) & 1, j = tid >> 6;
    const int u = 64 * j + 32 * cn + acc_row(i, hh);
    par[2 * C + 2 * tid] = ldexpf(1.f, -e1[u]);
    par[2 * C + 2 * tid + 1] = b1[u];
  }
  if (tid < C) {  // fc2 entry tid = (b * 2 + h) * 16 + i
    const int i = tid & 15, hh = (tid >> 4) & 1, b = tid >> 5;
    const int c = 32 * b + acc_row(i, hh);
    par[10 * C + 2 * tid] = ldexpf(1.f, -e2[c]);
    par[10 * C + 2 * tid + 1] = b2[c];
  }
  if (tid == 0) {  // max row norm of W1, max |b1| (one thread: 4C <= 1024 values each)
    float mn = 0.f, mb = 0.f;
    for (int u = 0; u < 4 * C; ++u) {
      mn = fmaxf(mn, n1[u]);
      mb = fmaxf(mb, fabsf(b1[u]));
    }
    par[12 * C] = mn;
    par[12 * C + 1] = mb;
    par[12 * C + 2] = 0.f;
    par[12 * C + 3] = 0.f;
  }
  (void)G::NB;
}

template <int C>
int pack_impl(const float* w1, const float* b1, const float* w2, const float* b2, const float* gamma,
              const float* beta, float* stream, float* par, int* ws, hipStream_t st) {
  int* e1 = ws;
  int* e2 = ws + 4 * C;
  float* n1 = reinterpret_cast<float*>(ws + 5 * C);
  mlp_rowstats_kernel<<<sfx::ceil_div(4 * C, 4), 256, 0, st>>>(4 * C, C, w1, e1, n1);
  mlp_rowstats_kernel<<<sfx::ceil_div(C, 4), 256, 0, st>>>(C, 4 * C, w2, e2, nullptr);
  const long long total = (long long)MlpGeom<C>::NCH * 2 * MlpGeom<C>::NB * 2048;
  mlp_pack_stream_kernel<C><<<sfx::ceil_div(total, 256), 256, 0, st>>>(w1, w2, e1, e2, stream);
  mlp_pack_params_kernel<C><<<sfx::ceil_div(4 * C, 256), 256, 0, st>>>(gamma, beta, b1, b2, e1, e2, n1, par);
  return sfx::check_launch("sfx_mlp_pack");
}

template <int C, int WAVES, int RING, bool HS = false, int KIND = MLP_EVAL, bool ONE = false>
int run_impl(int M, const float* x, long long ldx, const float* stream, const float* par, float eps, float* y,
             long long ldy, hipStream_t st, const float* rowscale = nullptr, float* z = nullptr) {
  static int rot = -1;
  if (rot < 0) {
    const char* e = getenv("SFX_MLP_ROT");
    rot = (e && *e) ? (atoi(e) != 0) : 1;
  }
  mlp_kernel<C, WAVES, RING, HS, KIND, ONE><<<sfx::ceil_div(M, HS ? WAVES * 16 : WAVES * 32), WAVES * 64, 0, st>>>(
      M, x, ldx, stream, par, eps, y, ldy, rot, rowscale, z);
  return sfx::check_launch(KIND == MLP_EVAL ? "sfx_block_mlp" : KIND == MLP_TRAIN ? "sfx_block_mlp_train"
                                                                                  : "sfx_block_mlp_bwd");
}

// The C = 256 eval tail split: one 4-wave workgroup per CU (512-register waves), so a launch of W workgroups runs
// ceil(W / CUs) rounds; when the last round is at most half full its workgroups run as SPLIT = 2 or 4 hidden-chunk
// splits (one round of 1/SPLIT the work) + mlp_combine_kernel.  Scratch: one buffer per (device, stream) behind a
// mutex (as sfx::lookback_state), grown on demand -- launches on two streams or host threads never share partials,
// and a stream's reuse is ordered by the stream itself.  Growing synchronises that stream before freeing the old
// buffer (work in flight may still read it), so it must not happen inside a graph capture: warm the entry up once
// at the captured sizes first (include/sfx.h, sfx_block_mlp).
float* mlp_split_scratch(size_t floats, hipStream_t st) {
  struct Buf {
    float* p = nullptr;
    size_t cap = 0;
  };
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, Buf> bufs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  Buf& b = bufs[{dev, st}];
  if (b.cap < floats) {
    if (b.p) {
      if (hipStreamSynchronize(st) != hipSuccess || hipFree(b.p) != hipSuccess) return nullptr;
      b = Buf();
    }
    void* q = nullptr;
    if (hipMalloc(&q, floats * sizeof(float)) != hipSuccess) return nullptr;
    b.p = static_cast<float*>(q);
    b.cap = floats;
  }
  return b.p;
}

int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

template <int C, int WAVES, int RING, bool HS, int KIND = MLP_EVAL, bool ONE = false>
int run_split(int M, const float* x, long long ldx, const float* stream, const float* par, float eps, float* y,
              long long ldy, hipStream_t st, const float* rowscale, float* z) {
  constexpr int PTS = HS ? WAVES * 16 : WAVES * 32;  // points per workgroup
  constexpr int NCH = C / 16;                       // hidden chunks
  const int wgs = (M + PTS - 1) / PTS, slots = ((WAVES == 4 && C > 128) ? 1 : 2) * cu_count();
  const int full = wgs / slots * slots, r = wgs - full;
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("SFX_MLP_SPLIT");
    mode = (e && *e) ? atoi(e) : 1;
  }
  int S = 1;
  // (the 128-point non-HS launches of C <= 96 measured no gain: their rounds are short and the combine is not free)
  if (HS && mode && full > 0 && r > 0) {
    for (int cand : {4, 3, 2})
      if (NCH % cand == 0 && cand * r <= slots) { S = cand; break; }
  }
  if (S == 1) return run_impl<C, WAVES, RING, HS, KIND, ONE>(M, x, ldx, stream, par, eps, y, ldy, st, rowscale, z);
  const int M1 = full * PTS, Mt = M - M1;
  float* P = mlp_split_scratch((size_t)S * Mt * C, st);
  SFX_REQUIRE(P, "sfx_block_mlp: tail scratch allocation failed");
  int rc = run_impl<C, WAVES, RING, HS, KIND, ONE>(M1, x, ldx, stream, par, eps, y, ldy, st, rowscale, z);
  if (rc) return rc;
  const float* xt = x + (size_t)M1 * ldx;
  float* yt = y + (size_t)M1 * ldy;
  const float* rst = rowscale ? rowscale + M1 : nullptr;
  // EVAL: z is the optional row-exponent output (written by the combine); TRAIN / BWD: the [M, 4C] pre-activation
  int* et = (KIND == MLP_EVAL && z) ? reinterpret_cast<int*>(z) + M1 : nullptr;
  float* zt = (KIND != MLP_EVAL) ? z + (size_t)M1 * 4 * C : nullptr;
  const dim3 grid((unsigned)r, (unsigned)S);
#define SFX_MLP_SPLIT_LAUNCH(SS)                                                                                   \
  do {                                                                                                            \
    mlp_kernel<C, WAVES, RING, HS, KIND, ONE, SS><<<grid, WAVES * 64, 0, st>>>(Mt, xt, ldx, stream, par, eps, yt, \
                                                                               ldy, 1, rst, zt, P);             \
    mlp_combine_kernel<SS><<<(unsigned)((Mt + 3) / 4), 256, 0, st>>>(Mt, C, KIND == MLP_BWD ? nullptr : xt, ldx, P, \
                                                                     yt, ldy, et);                               \
  } while (0)
  if constexpr (NCH % 4 == 0) { if (S == 4) SFX_MLP_SPLIT_LAUNCH(4); }
  if constexpr (NCH % 3 == 0) { if (S == 3) SFX_MLP_SPLIT_LAUNCH(3); }
  if constexpr (NCH % 2 == 0) { if (S == 2) SFX_MLP_SPLIT_LAUNCH(2); }
#undef SFX_MLP_SPLIT_LAUNCH
  return sfx::check_launch("sfx_block_mlp (split tail)");
}

template <int C, int WAVES, int RING, bool HS>
int run_eval_split(int M, const float* x, long long ldx, const float* stream, const float* par, float eps, float* y,
                   long long ldy, hipStream_t st, int* rowexp) {
  return run_split<C, WAVES, RING, HS>(M, x, ldx, stream, par, eps, y, ldy, st, nullptr,
                                       reinterpret_cast<float*>(rowexp));
}

// the training kinds run the default eval geometry of each C (4 waves; hidden split at C = 128, 256, and for the
// C = 96 backward, whose whole-chunk tile spills)
template <int KIND, bool ONE>
int run_train_p(int M, int C, const float* x, long long ldx, const float* stream, const float* par, float eps, float* y,
                long long ldy, hipStream_t st, const float* rowscale, float* z) {
  switch (C) {
    case 64: return run_impl<64, 4, 4, false, KIND, ONE>(M, x, ldx, stream, par, eps, y, ldy, st, rowscale, z);
    case 96:
      return run_impl<96, 4, 4, KIND == MLP_BWD, KIND, ONE>(M, x, ldx, stream, par, eps, y, ldy, st, rowscale, z);
    case 128: return run_split<128, 4, 4, true, KIND, ONE>(M, x, ldx, stream, par, eps, y, ldy, st, rowscale, z);
    default:
      return run_split<256, 4, SFX_MLP_RING256, true, KIND, ONE>(M, x, ldx, stream, par, eps, y, ldy, st, rowscale, z);
  }
}

template <int KIND>
int run_train(int M, int C, const float* x, long long ldx, const float* stream, const float* par, float eps, float* y,
              long long ldy, hipStream_t st, const float* rowscale, float* z) {
  return sfx_get_precision() == 1
             ? run_train_p<KIND, true>(M, C, x, ldx, stream, par, eps, y, ldy, st, rowscale, z)
             : run_train_p<KIND, false>(M, C, x, ldx, stream, par, eps, y, ldy, st, rowscale, z);
}

inline bool mlp_channels_ok(int C) { return C == 64 || C == 96 || C == 128 || C == 256; }

int check_mlp_args(const char* what, int M, int C, const float* x, long long ldx, const float* stream,
                   const float* params, const float* y, long long ldy, const float* z) {
  SFX_REQUIRE(M >= 0 && mlp_channels_ok(C), "%s: C must be one of 64, 96, 128, 256 (got %d)", what, C);
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(x && stream && params && y && z, "%s: null buffer", what);
  SFX_REQUIRE(ldx >= C && ldy >= C && ldx % 4 == 0 && ldy % 4 == 0, "%s: leading dimensions", what);
  SFX_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(z) |
                reinterpret_cast<uintptr_t>(stream) | reinterpret_cast<uintptr_t>(params)) & 15) == 0,
              "%s: buffers must be 16-byte aligned", what);
  SFX_REQUIRE((long long)M * ldx * 4 + 64 < (long long)OOB && (long long)M * ldy * 4 + 64 < (long long)OOB,
              "%s: operand exceeds the 2 GiB buffer-descriptor range", what);
  SFX_REQUIRE(x != y, "%s: in-place output is not supported", what);
  return SFX_OK;
}


}  // namespace

extern "C" {

size_t sfx_mlp_stream_floats(int C) { return mlp_channels_ok(C) ? (size_t)8 * C * C : 0; }
size_t sfx_mlp_params_floats(int C) { return mlp_channels_ok(C) ? (size_t)(12 * C + 4) : 0; }

int sfx_mlp_pack(int C, const float* w1, const float* b1, const float* w2, const float* b2, const float* gamma,
                 const float* beta, float* stream, float* params, int* workspace, void* stream_) {
  SFX_REQUIRE(mlp_channels_ok(C), "sfx_mlp_pack: C must be one of 64, 96, 128, 256 (got %d)", C);
  SFX_REQUIRE(w1 && b1 && w2 && b2 && gamma && beta && stream && params && workspace, "sfx_mlp_pack: null buffer");
  hipStream_t st = sfx::as_stream(stream_);
  switch (C) {
    case 64: return pack_impl<64>(w1, b1, w2, b2, gamma, beta, stream, params, workspace, st);
    case 96: return pack_impl<96>(w1, b1, w2, b2, gamma, beta, stream, params, workspace, st);
    case 128: return pack_impl<128>(w1, b1, w2, b2, gamma, beta, stream, params, workspace, st);
    default: return pack_impl<256>(w1, b1, w2, b2, gamma, beta, stream, params, workspace, st);
  }
}

int sfx_block_mlp(int M, int C, const float* x, long long ldx, const float* stream, const float* params, float eps,
                  float* y, long long ldy, int* rowexp, void* stream_) {
  SFX_REQUIRE(M >= 0 && mlp_channels_ok(C), "sfx_block_mlp: C must be one of 64, 96, 128, 256 (got %d)", C);
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(x && stream && params && y, "sfx_block_mlp: null buffer");
  SFX_REQUIRE(ldx >= C && ldy >= C && ldx % 4 == 0 && ldy % 4 == 0, "sfx_block_mlp: leading dimensions");
  SFX_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                reinterpret_cast<uintptr_t>(stream) | reinterpret_cast<uintptr_t>(params)) & 15) == 0,
              "sfx_block_mlp: buffers must be 16-byte aligned");
  SFX_REQUIRE((long long)M * ldx * 4 + 64 < (long long)OOB && (long long)M * ldy * 4 + 64 < (long long)OOB,
              "sfx_block_mlp: operand exceeds the 2 GiB buffer-descriptor range");
  SFX_REQUIRE(x != y, "sfx_block_mlp: in-place output is not supported");
  hipStream_t st = sfx::as_stream(stream_);
  // C <= 128: 4-wave (128-point) workgroups, two per CU -- measured 1.0-1.2x faster than one 8-wave workgroup
  // (profiles/r04_mlp_waves_hs.txt); SFX_MLP_WAVES=8 restores the 256-point workgroups.  Hidden split (a wave pair
  // per 32 points): SFX_MLP_HS=1 (default) at C = 128 and 256, where it measured faster (108.8 -> 100.0 /
  // 239.7 -> 220.6 us); 2 at every C; 0 nowhere.  Both read per call (tests switch them).
  const char* e = getenv("SFX_MLP_WAVES");
  const int waves = (e && *e) ? atoi(e) : 4;
  const char* f = getenv("SFX_MLP_HS");
  const int hs = (f && *f) ? atoi(f) : 1;
  switch (C) {
    // (waves, ring phases): 4 waves = 128 points per workgroup, 2 workgroups per CU for C <= 128 (64 KB ring);
    // C = 256 runs 4 waves as 2 hidden-split pairs (its LN2 fragments + output accumulators fill 512 registers)
    case 64: return waves == 4 ? (hs == 2 ? run_impl<64, 4, 4, true>(M, x, ldx, stream, params, eps, y, ldy, st, nullptr, reinterpret_cast<float*>(rowexp))
                                          : run_eval_split<64, 4, 4, false>(M, x, ldx, stream, params, eps, y, ldy, st, rowexp))
                               : run_impl<64, 8, 4>(M, x, ldx, stream, params, eps, y, ldy, st, nullptr, reinterpret_cast<float*>(rowexp));
    case 96: return waves == 4 ? (hs == 2 ? run_impl<96, 4, 4, true>(M, x, ldx, stream, params, eps, y, ldy, st, nullptr, reinterpret_cast<float*>(rowexp))
                                          : run_eval_split<96, 4, 4, false>(M, x, ldx, stream, params, eps, y, ldy, st, rowexp))
                               : run_impl<96, 8, 4>(M, x, ldx, stream, params, eps, y, ldy, st, nullptr, reinterpret_cast<float*>(rowexp));
    case 128: return waves == 4 ? (hs >= 1 ? run_eval_split<128, 4, 4, true>(M, x, ldx, stream, params, eps, y, ldy, st, rowexp)
                                          : run_impl<128, 4, 4>(M, x, ldx, stream, params, eps, y, ldy, st, nullptr, reinterpret_cast<float*>(rowexp)))
                                : run_impl<128, 8, 4>(M, x, ldx, stream, params, eps, y, ldy, st, nullptr, reinterpret_cast<float*>(rowexp));
    default: return hs ? run_eval_split<256, 4, SFX_MLP_RING256, true>(M, x, ldx, stream, params, eps, y, ldy, st, rowexp)
                       : run_impl<256, 4, SFX_MLP_RING256>(M, x, ldx, stream, params, eps, y, ldy, st, nullptr, reinterpret_cast<float*>(rowexp));
  }
}

// (ABI v13) training forward: as sfx_block_mlp, plus z [M, 4C] (contiguous) = the pre-activation fc1(LN2(x)) and
// the DropPath keep factor rowscale [M] (NULL: 1) on the branch: y = x + rowscale * (fc2(GELU(z)) + b2)
int sfx_block_mlp_train(int M, int C, const float* x, long long ldx, const float* stream, const float* params,
                        float eps, const float* rowscale, float* z, float* y, long long ldy, void* stream_) {
  const int rc = check_mlp_args("sfx_block_mlp_train", M, C, x, ldx, stream, params, y, ldy, z);
  if (rc != SFX_OK || M == 0) return rc;
  return run_train<MLP_TRAIN>(M, C, x, ldx, stream, params, eps, y, ldy, sfx::as_stream(stream_), rowscale, z);
}

// (ABI v13) training backward of the branch: dh2 = W1^T (GELU'(z) o W2^T (rowscale * dy)) (LN2's backward and the
// residual are the caller's); stream / params from sfx_mlp_pack(C, W2^T, 0, W1^T, 0, gamma, beta) -- the
// transposed weights in fc1's / fc2's places, zero biases
int sfx_block_mlp_bwd(int M, int C, const float* dy, long long lddy, const float* stream, const float* params,
                      const float* rowscale, const float* z, float* dh2, long long lddh, void* stream_) {
  const int rc = check_mlp_args("sfx_block_mlp_bwd", M, C, dy, lddy, stream, params, dh2, lddh, z);
  if (rc != SFX_OK || M == 0) return rc;
  return run_train<MLP_BWD>(M, C, dy, lddy, stream, params, 0.f, dh2, lddh, sfx::as_stream(stream_), rowscale,
                            const_cast<float*>(z));
}

}  // extern "C"
