// Block.cpe + shortcut + norm1 of the eval forward in one launch, the SubM conv summed in MFMA registers
// (reference calflops.py:45-53: x1 = x + LN_cpe(Linear(SubMConv3d(x))); h = norm1(x1); spconv SubMConv3d k = 3,
// Pointcept Block.cpe -- SURVEY A.1.7):
//
//   x1 = x + LN_cpe(b' + sum_k W'_k x_{nbr(i,k)}),   h = LN1(x1)
//
// with the CPE Linear folded into the conv (W'_k = W_lin W_k, b' = W_lin b_conv + b_lin; ptv3.Block.cpe_fused).
//
// Output-row stationary implicit GEMM: a wave owns 32 output points (two 16-point groups) and ALL C output
// channels; their conv sums live in MFMA accumulators for all 27 offsets, so no partial row ever leaves the chip
// (the offset-major pair GEMM this replaces stored one fp32 row per (offset, output) pair and a LayerNorm kernel
// read them back: 2.9x the algorithmic HBM bytes of a config-B refine).
//
// * Rows are processed in a per-map order (sfx_subm_order_keys + a radix sort, once per SubM map, shared by every
//   conv of the stage): rows sorted by 16 bits of their neighbour mask, rarer offsets (corners, edges) in the
//   key's high bits, so a 16-point group's rows mostly share their active offsets.  The order only decides which
//   rows share a group: a point's sum is the same bit for bit in any order (a missing neighbour adds exact zeros).  A (group, offset) with no
//   neighbour is skipped (wave-uniform branch); a partly active one gathers zero rows for its missing points
//   (measured on the config-B scene: 1.52-1.85x the pair products at 16-point granularity).
// * Computed transposed (points on the B side): D[16 channels x 16 points] += W'_k[16 x 32] . X^T[32 x 16] on
//   v_mfma_f32_16x16x32_f16, fp32-accurate fp16x2 terms (h*h + h*l + l*h, smallest first, as the GEMM family).
//   Scales: W' rows (output channels) by their max over all 27 offsets (sfx_subm_cpe_pack); a point's gathered
//   rows all by ONE power of two, the min over its neighbours' row exponents (sfx_subm_rowexp: the row maximum in
//   [2^14, 2^15)), so the 27 offsets accumulate on one scale and the epilogue unscales exactly.
// * W'_k streams through an LDS ring by LDS-DMA (global_load_lds_dwordx4) in exact fragment order (sfx_subm_cpe_pack
//   lays out [k][k-step][16-channel block][term][lane] x 16 B, so a slab is a plain copy and every fragment read is
//   a conflict-free contiguous ds_read_b128); only the offsets some group of the workgroup needs are streamed.
//   One raw barrier per phase, counted vmcnt (the gathers are issued unconditionally -- out-of-range offsets read
//   0 -- so every wait count is a compile-time constant).
// * The gathered neighbour rows go straight to registers (buffer loads of each lane's B-fragment channels; absent
//   neighbours read out of range = 0), PD k-steps ahead of their use.
// * Epilogue per point (4 lanes share a point): unscale + b' -> LN_cpe -> + x -> LN1, written to the point's row.
#include <cstdlib>

#pragma clang diagnostic ignored "-Winline-asm"  // dma16 clobbers M0 (see there)

#include "gemm_common.h"

namespace {

using namespace sfxg;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

constexpr int FRAG_BYTES = 2048;  // one 16-channel output block of one k-step: 2 terms x 64 lanes x 16 B

template <int C, int BPP>
struct OsGeom {
  static constexpr int NB = C / 16;               // 16-channel output blocks
  static constexpr int NS = C / 32;               // 32-channel input k-steps per offset
  static constexpr int NBP = NB > BPP ? BPP : NB;  // output blocks per ring phase
  static constexpr int NCH = NB / NBP;            // phases per k-step
  static constexpr int PHASE = NBP * FRAG_BYTES;  // bytes per ring phase
  static_assert(NB % NBP == 0, "phase split");
};

template <int N>
__device__ __forceinline__ void wait_vm_lgkm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One LDS-DMA piece (16 B per lane from its own global address to M0 + 16 lane) in inline asm: the builtin makes the
// compiler drain vmcnt to 0 whenever an address register is reused (serialising every DMA behind the previous
// one) and treat every later LDS read as aliasing it; here the compiler sees no VMEM op and every wait is ours.
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds_dst) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_dst) : "memory", "m0");
}

// timing stamps (SFX_SUBM_OS_DEBUG bit 4: workgroup 0 only; diagnostics, never read by the computation)
__device__ unsigned long long g_os_stamps[2][1024];
#define OS_STAMP(slot)                                                                                        \
  do {                                                                                                        \
    if ((dbg & 16) && blockIdx.x == 0 && (wid == 0 || wid == LW) && lane == 0 && (slot) < 1024)              \
      g_os_stamps[wid == 0 ? 0 : 1][(slot)] = __builtin_amdgcn_s_memtime();                                   \
  } while (0)

// 32-bit LDS address of a pointer into a __shared__ array
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)(p));
}

__device__ __forceinline__ f16x8 pack8(uint2 a, uint2 b) {
  return __builtin_bit_cast(f16x8, make_uint4(a.x, a.y, b.x, b.y));
}

// One workgroup = LW loader waves + CW compute waves (runtime: blockDim.x / 64 - LW).  The loaders only stream W'
// into the LDS ring (PHASE / 1 KB / LW DMA pieces each per phase), so their vmcnt holds nothing else and the
// compute waves' holds only their own gathers, which the compiler then waits for exactly.  Compute wave w owns GPW
// 16-point groups, points 16 GPW w .. 16 GPW (w + 1) - 1 of the workgroup's rows perm[blockIdx.x * PTS ..].  Lane
// (q = lane >> 4, r = lane & 15) holds point r of each of the wave's groups -- its B fragment of k-step s is the
// point's channels 32 s + 8 q .. + 7 -- and accumulator rows 16 b + 4 q + i (i < 4) of every output block b.  A wave
// computes its groups together (GPW = 2: both, whenever one of them has a neighbour at the offset) and skips an
// offset none of its points has (wave-uniform branch; it still takes part in the ring protocol).
// RING: LDS phases; PD: k-steps of gathers in flight (registers); BPP: output blocks per phase.
// waves per workgroup at most: 16 (128 VGPRs) while the accumulators are small, 12 (168 VGPRs) from 256 channels
constexpr int os_maxw(int acc_channels) { return acc_channels >= 256 ? 12 : 16; }

template <int C, int GPW, int LW, int RING, int PD, int BPP>
struct OsCfg {
  using G = OsGeom<C, BPP>;
  static constexpr int PIECES = G::PHASE / (LW * 1024);    // per loader wave per phase
  static constexpr int GL = 2 * GPW;                        // gather loads per wave per k-step (2 per group)
  static constexpr int GATHER_OFF = RING * G::PHASE;        // then s_nbr, then s_kl
  static constexpr int MAXW = os_maxw(C * GPW);
  static_assert(G::PHASE % (LW * 1024) == 0, "phase pieces");
  static_assert(RING >= 3, "ring depth");
  static constexpr size_t lds_bytes(int cw) {
    return (size_t)GATHER_OFF + (size_t)cw * 16 * GPW * 27 * 4 + 32 * 4;
  }
};

template <int C, int GPW, int LW, int RING, int PD, int BPP>
__global__ void __launch_bounds__(64 * os_maxw(C * GPW))
    subm_cpe_ln_kernel(int n, const float* __restrict__ xc, const float* __restrict__ xres,
                       const int* __restrict__ nbr, const int* __restrict__ perm, const int* __restrict__ rowexp,
                       const float* __restrict__ wstream, const float* __restrict__ winv,
                       const float* __restrict__ bias, const float* __restrict__ g_cpe,
                       const float* __restrict__ b_cpe, const float* __restrict__ g1, const float* __restrict__ b1,
                       float eps, float* __restrict__ x1out, float* __restrict__ hout, int dbg) {
  using Q = OsCfg<C, GPW, LW, RING, PD, BPP>;
  using G = typename Q::G;
  constexpr int NB = G::NB, NS = G::NS, NBP = G::NBP, NCH = G::NCH, PHASE = G::PHASE;
  constexpr int PIECES = Q::PIECES, GL = Q::GL;
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: role branches are scalar
  const int CW = (int)(blockDim.x >> 6) - LW, NTH = (int)blockDim.x;
  const int PTS = CW * 16 * GPW;
  const int q = lane >> 4, r16 = lane & 15;
  const int base = (int)blockIdx.x * PTS;
  const bool loader = wid < LW;
  const int cw = wid - LW;  // compute wave index
  int* s_nbr = reinterpret_cast<int*>(lds + Q::GATHER_OFF);  // [PTS][27]
  int* s_kl = s_nbr + PTS * 27;  // [28]: the workgroup's union offset mask

  // ---- prologue: neighbour rows, per-point mask / scale, per-wave masks, workgroup offset list ----
  for (int e = tid; e < PTS * 27; e += NTH) {
    const int j = e / 27, k = e - 27 * j;
    const int P = base + j;
    s_nbr[e] = P < n ? nbr[27ll * perm[P] + k] : -1;
  }
  if (tid == 0) s_kl[28] = 0;
  __syncthreads();
  int orow[GPW], ep[GPW];
  unsigned wm = 0;  // offsets some point of this wave has
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    if (loader) {
      orow[g] = -1;
      ep[g] = 0;
      continue;
    }
    const int j = 16 * (GPW * cw + g) + r16;
    const int P = base + j;
    orow[g] = P < n ? perm[P] : -1;
    unsigned m = 0;
    int e = 127;
    for (int k = q; k < 27; k += 4) {
      const int src = s_nbr[j * 27 + k];
      if (src >= 0) {
        m |= 1u << k;
        e = min(e, rowexp[src]);
      }
    }
    m |= __shfl_xor(m, 16, 64);
    m |= __shfl_xor(m, 32, 64);
    e = min(e, __shfl_xor(e, 16, 64));
    e = min(e, __shfl_xor(e, 32, 64));
    ep[g] = e > 126 ? 0 : e;  // no neighbour row with a non-zero value: any scale
    wm |= m;
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) wm |= __shfl_xor(wm, o, 64);
  wm = __builtin_amdgcn_readfirstlane(wm);
  if (lane == 0) atomicOr(reinterpret_cast<unsigned*>(&s_kl[28]), wm);
  __syncthreads();
  const unsigned uni = __builtin_amdgcn_readfirstlane((unsigned)s_kl[28]);
  OS_STAMP(0);
  const int nks = __popc(uni) * NS;  // k-steps of this workgroup
  const int NP = nks * NCH;           // ring phases

  // ---- streams: W' phases by LDS-DMA (inline asm), gathered rows into registers (compiler-visible loads) ----
  // Three cursors walk the workgroup's offsets (ascending set bits of `uni`) in scalar registers.
  struct Cursor {
    unsigned rem;  // offsets not reached yet
    int k, s, c;   // offset (27: past the end), k-step within it, phase within the k-step
  };
  auto cursor0 = [&]() {
    Cursor x;
    x.k = uni ? (int)__builtin_ctz(uni) : 27;
    x.rem = uni & (uni - 1u);
    x.s = 0;
    x.c = 0;
    return x;
  };
  auto next_kstep = [&](Cursor& x) {
    if (++x.s == NS) {
      x.s = 0;
      x.k = x.rem ? (int)__builtin_ctz(x.rem) : 27;
      x.rem &= x.rem - 1u;
    }
  };
  auto next_phase = [&](Cursor& x) {
    if (++x.c == NCH) {
      x.c = 0;
      next_kstep(x);
    }
  };
  const char* gw = reinterpret_cast<const char*>(wstream);
  Cursor dcur = cursor0();  // next W' phase to stream
  int dslot = 0;            // its ring slot
  const unsigned lds0 = lds_addr(lds);
  auto issue_dma = [&]() {  // loader waves only
    if (!(dbg & 4)) {
      const char* src = gw + ((size_t)((dcur.k * NS + dcur.s) * NB + dcur.c * NBP)) * FRAG_BYTES +
                        wid * (PIECES * 1024) + lane * 16;
      const unsigned dst = lds0 + dslot * PHASE + wid * (PIECES * 1024);
#pragma unroll
      for (int pc = 0; pc < PIECES; ++pc) dma16(src + pc * 1024, __builtin_amdgcn_readfirstlane(dst + pc * 1024));
    }
    next_phase(dcur);
    dslot = dslot + 1 == RING ? 0 : dslot + 1;
  };
  // k-step t's gathered rows go to raw[t % PD]: lane (q, r) loads channels 32 s + 8 q .. + 7 of point r of each
  // group -- its B fragment.  Issued for every k-step (an out-of-range read = 0 where the point has no neighbour,
  // the wave none at all, or past the last k-step); the neighbour row of each group is read from LDS once per
  // offset.  The compiler waits for these registers itself (it sees no DMA: the W' DMAs are inline asm).
  const __amdgpu_buffer_rsrc_t rX = rsrc_ext(xc, (unsigned)n * (unsigned)C * 4u);
  Cursor gcur = cursor0();  // next k-step to gather
  int gsrc[GPW];            // its neighbour rows (-1: none)
  auto gather_rows = [&]() {
    const bool wact = gcur.k < 27 && ((wm >> gcur.k) & 1u) && !(dbg & 2);
#pragma unroll
    for (int g = 0; g < GPW; ++g) gsrc[g] = wact ? s_nbr[(16 * (GPW * cw + g) + r16) * 27 + gcur.k] : -1;
  };
  float4 raw[PD][GPW][2];
  auto issue_gather = [&](float4 (&v)[GPW][2]) {
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      const unsigned off =
          gsrc[g] >= 0 ? ((unsigned)gsrc[g] * (unsigned)C + (unsigned)(32 * gcur.s + 8 * q)) * 4u : OOB;
      v[g][0] = bload4(rX, off);
      v[g][1] = bload4(rX, gsrc[g] >= 0 ? off + 16u : OOB);
    }
    if (gcur.k < 27) {
      next_kstep(gcur);
      if (gcur.s == 0) gather_rows();
    }
  };
  float sc[GPW];
#pragma unroll
  for (int g = 0; g < GPW; ++g) sc[g] = ldexpf(1.f, ep[g]);
  f16x8 bh[GPW], bl[GPW];    // the B fragments of the k-step being computed
  f16x8 nbh[GPW], nbl[GPW];  // ... and of the next one (prepared during this one's last phase)
  // split unconditionally (a wave with no neighbour at the offset skips the MFMAs, not this): a branch here would
  // make the compiler drain vmcnt at its join before the next gathers overwrite the registers
  auto prep = [&](const float4 (&v)[GPW][2]) {
#pragma unroll
    for (int g = 0; g < GPW; ++g) {
      uint2 a2[2], b2[2];
      sfx::split2h(v[g][0], sc[g], a2);
      sfx::split2h(v[g][1], sc[g], b2);
      nbh[g] = pack8(a2[0], b2[0]);
      nbl[g] = pack8(a2[1], b2[1]);
    }
  };
  if (loader) {  // ---- loader waves: the W' ring, one barrier per phase like the compute waves ----
#pragma unroll
    for (int p = 0; p < RING - 1; ++p)
      if (p < NP) issue_dma();
#pragma unroll 1
    for (int p = 0; p < NP; ++p) {
      // DMA(p) has the RING - 2 later phases' DMAs younger than it (nothing else in this wave's vmcnt)
      OS_STAMP(4 + 4 * p);
      if (p + RING - 1 < NP) wait_vm_lgkm<(RING - 2) * PIECES>();
      else wait_vm_lgkm<0>();
      OS_STAMP(5 + 4 * p);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      OS_STAMP(6 + 4 * p);
      if (p + RING - 1 < NP) issue_dma();  // into the slot every wave finished reading before this barrier
      OS_STAMP(7 + 4 * p);
    }
    return;
  }
  gather_rows();
#pragma unroll
  for (int u = 0; u < PD; ++u) issue_gather(raw[u]);
  Cursor ccur = cursor0();  // the k-step being computed
  prep(raw[0]);  // k-step 0's fragments
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    bh[g] = nbh[g];
    bl[g] = nbl[g];
  }
  issue_gather(raw[0]);  // k-step PD's rows into the freed slot

  f32x4 acc[GPW][NB];
#pragma unroll
  for (int g = 0; g < GPW; ++g)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[g][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- compute waves: per phase p: [barrier] [MFMAs of phase p] [last phase of a k-step: the next k-step's
  // fragments from its gathered registers, the gathers of k-step t + 1 + PD].  The MFMAs come first so a wave's
  // split VALU and load issue overlap the other waves' MFMAs.
  int p = 0, rslot = 0;
#pragma unroll 1
  for (int t0 = 0; t0 < nks; t0 += PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int t = t0 + u;
      if (t < nks) {
        const int k = ccur.k;
        next_kstep(ccur);
        const bool wact = (wm >> k) & 1u;
#pragma unroll
        for (int c = 0; c < NCH; ++c, ++p) {
          OS_STAMP(4 + 4 * p);
          wait_vm_lgkm<63>();  // lgkmcnt(0): this wave's reads of the slot refilled after the barrier returned
          OS_STAMP(5 + 4 * p);
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          OS_STAMP(6 + 4 * p);
          const bool lastc = c == NCH - 1;  // k-step t + 1's fragments are prepared in this phase
          const int un = (u + 1) % PD;
          if (wact && !(dbg & 1)) {
            const char* ph = lds + rslot * PHASE + lane * 16;
            f16x8 fa[2][2];  // [pipeline stage][term]: block b + 1's fragments are read during block b's MFMAs
            fa[0][0] = *reinterpret_cast<const f16x8*>(ph);
            fa[0][1] = *reinterpret_cast<const f16x8*>(ph + 1024);
#pragma unroll
            for (int b = 0; b < NBP; ++b) {
              if (b + 1 < NBP) {
                fa[(b + 1) & 1][0] = *reinterpret_cast<const f16x8*>(ph + (b + 1) * FRAG_BYTES);
                fa[(b + 1) & 1][1] = *reinterpret_cast<const f16x8*>(ph + (b + 1) * FRAG_BYTES + 1024);
              }
              // the next k-step's split in the middle of this one's MFMAs (same basic block: its VALU issues in
              // the MFMAs' shadow instead of after them)
              if (C >= 128 && lastc && b == NBP / 2) prep(raw[un]);  // (C < 128: measured slower, after)
              const f16x8 ah = fa[b & 1][0], al = fa[b & 1][1];
#pragma unroll
              for (int g = 0; g < GPW; ++g) {
                f32x4& a = acc[g][c * NBP + b];
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[g], a, 0, 0, 0);  // smallest terms first
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[g], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[g], a, 0, 0, 0);
              }
            }
          }
          if (lastc && (C < 128 || !(wact && !(dbg & 1)))) prep(raw[un]);
          OS_STAMP(7 + 4 * p);
          if (lastc) {  // the prepared fragments become current; k-step t + 1 + PD's rows into the freed slot
#pragma unroll
            for (int g = 0; g < GPW; ++g) {
              bh[g] = nbh[g];
              bl[g] = nbl[g];
            }
            issue_gather(raw[un]);
          }
          rslot = rslot + 1 == RING ? 0 : rslot + 1;
        }
      }
    }
  }
  OS_STAMP(1);
  wait_vm<0>();  // the trailing (zero-row) gathers
  OS_STAMP(2);
  if (dbg & 8) return;

  // ---- epilogue: t = acc / (s_o s_p) + b' -> LN_cpe -> + x -> LN1, per point (4 lanes: xor 16, 32) ----
  const __amdgpu_buffer_rsrc_t rR = rsrc_ext(xres, (unsigned)n * (unsigned)C * 4u);
  const __amdgpu_buffer_rsrc_t rO = rsrc_ext(x1out, (unsigned)n * (unsigned)C * 4u);
  const __amdgpu_buffer_rsrc_t rH = rsrc_ext(hout, (unsigned)n * (unsigned)C * 4u);
  const float inv_c = 1.f / (float)C;
#pragma unroll
  for (int g = 0; g < GPW; ++g) {
    const float sinv = ldexpf(1.f, -ep[g]);
    float s1 = 0.f;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int c0 = 16 * b + 4 * q;
      asm volatile("" ::: "memory");  // one block's parameters at a time: the accumulators hold the registers
      const float4 wi = *reinterpret_cast<const float4*>(winv + c0);
      const float4 bi = *reinterpret_cast<const float4*>(bias + c0);
      acc[g][b][0] = acc[g][b][0] * (wi.x * sinv) + bi.x;
      acc[g][b][1] = acc[g][b][1] * (wi.y * sinv) + bi.y;
      acc[g][b][2] = acc[g][b][2] * (wi.z * sinv) + bi.z;
      acc[g][b][3] = acc[g][b][3] * (wi.w * sinv) + bi.w;
      s1 += (acc[g][b][0] + acc[g][b][1]) + (acc[g][b][2] + acc[g][b][3]);
    }
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    const float mean = s1 * inv_c;
    float v1 = 0.f;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = acc[g][b][i] - mean;
        v1 += d * d;
      }
    v1 += __shfl_xor(v1, 16, 64);
    v1 += __shfl_xor(v1, 32, 64);
    const float rstd = 1.f / sqrtf(v1 * inv_c + eps);
    const unsigned rowoff = orow[g] >= 0 ? (unsigned)orow[g] * (unsigned)C * 4u : OOB;
    float s2 = 0.f;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int c0 = 16 * b + 4 * q;
      asm volatile("" ::: "memory");
      const float4 gg = *reinterpret_cast<const float4*>(g_cpe + c0);
      const float4 bb = *reinterpret_cast<const float4*>(b_cpe + c0);
      const float4 x = bload4(rR, rowoff == OOB ? OOB : rowoff + 4u * c0);
      acc[g][b][0] = x.x + ((acc[g][b][0] - mean) * rstd * gg.x + bb.x);
      acc[g][b][1] = x.y + ((acc[g][b][1] - mean) * rstd * gg.y + bb.y);
      acc[g][b][2] = x.z + ((acc[g][b][2] - mean) * rstd * gg.z + bb.z);
      acc[g][b][3] = x.w + ((acc[g][b][3] - mean) * rstd * gg.w + bb.w);
      s2 += (acc[g][b][0] + acc[g][b][1]) + (acc[g][b][2] + acc[g][b][3]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[g][b]), rO,
                                             rowoff == OOB ? OOB : rowoff + 4u * c0, 0, 0);
    }
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    const float mean2 = s2 * inv_c;
    float v2 = 0.f;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = acc[g][b][i] - mean2;
        v2 += d * d;
      }
    v2 += __shfl_xor(v2, 16, 64);
    v2 += __shfl_xor(v2, 32, 64);
    const float rstd2 = 1.f / sqrtf(v2 * inv_c + eps);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int c0 = 16 * b + 4 * q;
      asm volatile("" ::: "memory");
      const float4 gg = *reinterpret_cast<const float4*>(g1 + c0);
      const float4 bb = *reinterpret_cast<const float4*>(b1 + c0);
      f32x4 o;
      o[0] = (acc[g][b][0] - mean2) * rstd2 * gg.x + bb.x;
      o[1] = (acc[g][b][1] - mean2) * rstd2 * gg.y + bb.y;
      o[2] = (acc[g][b][2] - mean2) * rstd2 * gg.z + bb.z;
      o[3] = (acc[g][b][3] - mean2) * rstd2 * gg.w + bb.w;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), rH,
                                             rowoff == OOB ? OOB : rowoff + 4u * c0, 0, 0);
    }
  }
  OS_STAMP(3);
}

// ---- per-row exponents of the conv input: x_j * 2^e_j has its maximum in [2^14, 2^15) (127: an all-zero row) ----
__global__ void __launch_bounds__(256) subm_rowexp_kernel(int n, int C, const float* __restrict__ x,
                                                          int* __restrict__ e_out) {
  const int row = (int)blockIdx.x * 16 + (int)(threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  float m = 0.f;
  if (row < n)
    for (int c = 4 * sub; c < C; c += 64) {
      const float4 v = *reinterpret_cast<const float4*>(x + (long long)row * C + c);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (sub == 0 && row < n) {
    int e = 127;
    if (m > 0.f && m <= 3.4028235e38f) {
      e = 15 - __builtin_amdgcn_frexp_expf(m);  // m in [2^(e'-1), 2^e')
      e = e > 126 ? 126 : (e < -126 ? -126 : e);
    } else if (!(m <= 3.4028235e38f)) {
      e = 0;  // inf / nan: unscaled (propagates)
    }
    e_out[row] = e;
  }
}

// ---- row order of a SubM map: a 16-bit key of the neighbour mask, sorted by two 8-bit radix passes ----
// The key bits (high -> low) are the offsets k (27 = the 3x3x3 taps, k = 9 (dx+1) + 3 (dy+1) + (dz+1)) picked greedily
// on the config-B scene for the least MFMA-weighted padding: 7 corners, 7 edges, 2 faces (all 26 neighbour bits
// order the rows only 9 % better -- 4 radix passes instead of 2)
__constant__ int kOrderBits[16] = {2, 6, 8, 18, 20, 24, 26, 1, 7, 9, 11, 15, 17, 23, 10, 12};
__global__ void __launch_bounds__(256) subm_order_keys_kernel(int n, const int* __restrict__ nbr,
                                                              unsigned long long* __restrict__ keys) {
  const int i = (int)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  unsigned key = 0;
#pragma unroll
  for (int b = 0; b < 16; ++b) key = (key << 1) | (nbr[27ll * i + kOrderBits[b]] >= 0 ? 1u : 0u);
  keys[i] = key;
}

// per output channel o of W' [C, 27 C]: the fp16x2 exponent of its whole row (max over every offset and input)
__global__ void __launch_bounds__(64) subm_cpe_wscale_kernel(int C, const float* __restrict__ w,
                                                             float* __restrict__ winv, float* __restrict__ wsc) {
  const int o = blockIdx.x;
  float m = 0.f;
  for (int e = threadIdx.x; e < 27 * C; e += 64) m = fmaxf(m, fabsf(w[(long long)o * 27 * C + e]));
  m = sfx::wave_max(m);
  if (threadIdx.x == 0) {
    int e = 0;
    if (m > 0.f && m <= 3.4028235e38f) {
      e = 15 - __builtin_amdgcn_frexp_expf(m);
      e = e > 126 ? 126 : (e < -126 ? -126 : e);
    }
    wsc[o] = ldexpf(1.f, e);
    winv[o] = ldexpf(1.f, -e);
  }
}

// fragment stream: [k][k-step s][16-channel block b][term][lane] x 16 B; lane l holds
// W'[o = 16 b + (l & 15)][k C + 32 s + 8 (l >> 4) + j], j < 8, scaled by 2^e_o and split into fp16 h / l
__global__ void subm_cpe_pack_kernel(int C, const float* __restrict__ w, const float* __restrict__ wsc,
                                     uint4* __restrict__ wpk) {
  const int NB = C / 16, NS = C / 32;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // (k, s, b, lane)
  const long long total = 27ll * NS * NB * 64;
  if (t >= total) return;
  const int lane = (int)(t & 63);
  long long qq = t >> 6;
  const int b = (int)(qq % NB);
  qq /= NB;
  const int s = (int)(qq % NS);
  const int k = (int)(qq / NS);
  const int o = 16 * b + (lane & 15);
  const float* src = w + (long long)o * 27 * C + (long long)k * C + 32 * s + 8 * (lane >> 4);
  const float sc = wsc[o];
  uint2 a[2], c[2];
  sfx::split2h(make_float4(src[0], src[1], src[2], src[3]), sc, a);
  sfx::split2h(make_float4(src[4], src[5], src[6], src[7]), sc, c);
  const long long f = (((long long)k * NS + s) * NB + b) * 2;
  wpk[f * 64 + lane] = make_uint4(a[0].x, a[0].y, c[0].x, c[0].y);
  wpk[(f + 1) * 64 + lane] = make_uint4(a[1].x, a[1].y, c[1].x, c[1].y);
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline bool os_channels_ok(int C) { return C == 64 || C == 96 || C == 128 || C == 256; }

// One round of workgroups on the chip: the wave count per workgroup is the smallest that fits the rows into
// kCUs workgroups (>= LW loader waves, <= 16), so no second, mostly empty round of workgroups follows.
constexpr int kCUs = 256;
// SFX_SUBM_OS_DEBUG (timing ablations only, results wrong): bit 0 no MFMAs, 1 no gathers, 2 no W' DMAs, 3 no epilogue
inline int os_debug_flags() {
  static int f = -1;
  if (f < 0) {
    const char* e = getenv("SFX_SUBM_OS_DEBUG");
    f = (e && *e) ? atoi(e) : 0;
  }
  return f;
}
template <int C, int GPW, int LW, int RING, int PD, int BPP, int WPC = 1>
int launch(int n, const float* xc, const float* xres, const int* nbr, const int* perm, const int* rowexp,
           const void* wpk, const float* winv, const float* bias, const float* gc, const float* bc, const float* g1,
           const float* b1, float eps, float* x1, float* h, hipStream_t st) {
  using Q = OsCfg<C, GPW, LW, RING, PD, BPP>;
  int cw = (int)sfx::ceil_div(sfx::ceil_div(n, 16 * GPW), kCUs * WPC);  // compute waves (WPC workgroups per CU)
  cw = cw < 2 ? 2 : (cw > Q::MAXW - LW ? Q::MAXW - LW : cw);
  const int nw = LW + cw;
  const size_t lds = Q::lds_bytes(cw);
  SFX_REQUIRE(lds <= 163840, "sfx_subm_cpe_ln: %zu bytes of LDS for %d waves", lds, nw);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&subm_cpe_ln_kernel<C, GPW, LW, RING, PD, BPP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr_set = true;
  }
  if (os_debug_flags() & 16) {
    static unsigned long long zero[2][1024];
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_os_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice, st);
  }
  subm_cpe_ln_kernel<C, GPW, LW, RING, PD, BPP><<<sfx::ceil_div(n, 16 * GPW * cw), 64 * nw, lds, st>>>(
      n, xc, xres, nbr, perm, rowexp, reinterpret_cast<const float*>(wpk), winv, bias, gc, bc, g1, b1, eps, x1, h,
      os_debug_flags());
  if (os_debug_flags() & 16) {  // diagnostics: phase timeline of workgroup 0 (loader wave 0, non-loader wave LW)
    unsigned long long h[2][1024];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_os_stamps), sizeof(h));
    for (int w = 0; w < 2; ++w) {
      const unsigned long long t0 = h[w][0];
      fprintf(stderr, "[subm_os C=%d nw=%d wave %s] prologue->loop 0, loop end %lld, drain %lld, epilogue end %lld\n",
              C, nw, w ? "non-loader" : "loader", (long long)(h[w][1] - t0), (long long)(h[w][2] - t0),
              (long long)(h[w][3] - t0));
      for (int p = 0; p < 60 && h[w][4 + 4 * p]; ++p)
        fprintf(stderr, "  phase %2d: start %7lld wait %5lld barrier %5lld issue/bfrag %5lld\n", p,
                (long long)(h[w][4 + 4 * p] - t0), (long long)(h[w][5 + 4 * p] - h[w][4 + 4 * p]),
                (long long)(h[w][6 + 4 * p] - h[w][5 + 4 * p]), (long long)(h[w][7 + 4 * p] - h[w][6 + 4 * p]));
    }
  }
  return SFX_OK;
}

}  // namespace

extern "C" {

// bytes of the packed fp16x2 conv weight of sfx_subm_cpe_ln (0: C not served)
size_t sfx_subm_cpe_pack_bytes(int C) { return os_channels_ok(C) ? (size_t)27 * C * C * 4 : 0; }

// W' [C, 27*C] (row o = output channel, column k*C + i: the spconv [Cout, 3, 3, 3, Cin] layout with the CPE
// Linear folded in) -> fragment stream (sfx_subm_cpe_pack_bytes(C)) + inverse row scales winv[C] (ws: C floats)
int sfx_subm_cpe_pack(int C, const float* w, void* wpk, float* winv, float* ws, void* stream) {
  SFX_REQUIRE(os_channels_ok(C), "sfx_subm_cpe_pack: C must be 64, 96, 128 or 256 (got %d)", C);
  SFX_REQUIRE(w && wpk && winv && ws, "sfx_subm_cpe_pack: null buffer");
  SFX_REQUIRE(al16(wpk), "sfx_subm_cpe_pack: the stream must be 16-byte aligned");
  hipStream_t st = sfx::as_stream(stream);
  subm_cpe_wscale_kernel<<<C, 64, 0, st>>>(C, w, winv, ws);
  const long long total = 27ll * (C / 32) * (C / 16) * 64;
  subm_cpe_pack_kernel<<<sfx::ceil_div(total, 256), 256, 0, st>>>(C, w, ws, reinterpret_cast<uint4*>(wpk));
  return sfx::check_launch("sfx_subm_cpe_pack");
}

// sort keys of a SubM map's rows (sfx_subm_cpe_ln's row order = the argsort of these keys, bits [0, 16))
int sfx_subm_order_keys(int n, const int* nbr, uint64_t* keys, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_subm_order_keys: n < 0");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(nbr && keys, "sfx_subm_order_keys: null buffer");
  subm_order_keys_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(
      n, nbr, reinterpret_cast<unsigned long long*>(keys));
  return sfx::check_launch("sfx_subm_order_keys");
}

// per-row fp16x2 exponents of a conv input x [n, C] (contiguous rows)
int sfx_subm_rowexp(int n, int C, const float* x, int* e, void* stream) {
  SFX_REQUIRE(n >= 0 && C > 0 && C % 4 == 0, "sfx_subm_rowexp: bad shape (n %d, C %d)", n, C);
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(x && e && al16(x), "sfx_subm_rowexp: null or misaligned buffer");
  subm_rowexp_kernel<<<sfx::ceil_div(n, 16), 256, 0, sfx::as_stream(stream)>>>(n, C, x, e);
  return sfx::check_launch("sfx_subm_rowexp");
}

// x1 = xres + LN_cpe(bias + SubMConv'(xc)), h = LN1(x1) (see the top of this file); rows contiguous [n, C];
// perm: the map's row order (a permutation of 0..n-1), rowexp: sfx_subm_rowexp(xc)
int sfx_subm_cpe_ln(int n, int C, const float* xc, const float* xres, const int* nbr, const int* perm,
                    const int* rowexp, const void* wpk, const float* winv, const float* bias, const float* gamma_cpe,
                    const float* beta_cpe, const float* gamma1, const float* beta1, float eps, float* x_out,
                    float* h_out, void* stream) {
  SFX_REQUIRE(n >= 0 && os_channels_ok(C), "sfx_subm_cpe_ln: C must be 64, 96, 128 or 256 (got %d)", C);
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(xc && xres && nbr && perm && rowexp && wpk && winv && bias && gamma_cpe && beta_cpe && gamma1 &&
                  beta1 && x_out && h_out,
              "sfx_subm_cpe_ln: null buffer");
  SFX_REQUIRE(al16(xc) && al16(xres) && al16(wpk) && al16(winv) && al16(bias) && al16(gamma_cpe) &&
                  al16(beta_cpe) && al16(gamma1) && al16(beta1) && al16(x_out) && al16(h_out),
              "sfx_subm_cpe_ln: buffers must be 16-byte aligned");
  SFX_REQUIRE((long long)n * C * 4 + 64 < (long long)OOB, "sfx_subm_cpe_ln: rows exceed the buffer range");
  SFX_REQUIRE(x_out != xres && h_out != xres && x_out != xc && h_out != xc, "sfx_subm_cpe_ln: in-place output");
  hipStream_t st = sfx::as_stream(stream);
  int rc;
#define SFX_OS_ARGS n, xc, xres, nbr, perm, rowexp, wpk, winv, bias, gamma_cpe, beta_cpe, gamma1, beta1, eps, x_out, h_out, st
  // <C, groups per wave, loader waves, ring phases, gather k-steps in flight, output blocks per phase>
  switch (C) {
    case 64: rc = launch<64, 2, 2, 6, 2, 4>(SFX_OS_ARGS); break;
    case 96: rc = launch<96, 2, 2, 6, 2, 6>(SFX_OS_ARGS); break;
    case 128: rc = launch<128, 2, 2, 5, 2, 8>(SFX_OS_ARGS); break;
    default: rc = launch<256, 1, 2, 5, 2, 8>(SFX_OS_ARGS); break;
  }
#undef SFX_OS_ARGS
  if (rc != SFX_OK) return rc;
  return sfx::check_launch("sfx_subm_cpe_ln");
}

}  // extern "C"
