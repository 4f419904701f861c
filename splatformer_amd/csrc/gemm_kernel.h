// gemm_kernel.h -- the MFMA GEMM kernel template and its launcher; included only by the per-mode launcher
// translation units gemm_k<mode><waves>.hip (the instantiations compile in parallel).  Host-side dispatch, tile
// tables and the C-ABI entries are in gemm.hip.
//
// fp32 MFMA GEMM with fused gather prologue and bias/affine/act/residual
// epilogue -- the dense work of the PTv3 refiner (qkv/proj/MLP/CPE linears,
// embedding, pooling/unpooling projections, output heads) and the
// SubMConv3d CPE (centre offset as a gathered GEMM, the other 26 offsets as
// an offset-major pair GEMM with atomic accumulation).
//
//   Y[m, n] = act( (sum_k A'[m, k] W[n, k] + bias[n]) * scale[n] + shift[n] ) + R[r(m), n]
//
// A' is A (row-major, lda) or, with a gather index G (row stride gstride),
// the row concatenation of S segments of width Kseg: A'[m, s*Kseg + c] =
// A[G[m*gstride+s], c] (0 when G < 0).  W is torch's Linear layout [N, K].
//
// gfx950 mapping: v_mfma_f32_32x32x2_f32 (exact f32 FMA chains, 157 TF/s
// peak, no xf32 on CDNA4), 256 threads = 4 waves in a 2x2 grid, each wave a
// (BM/2)x(BN/2) sub-tile of 32x32 MFMA blocks; BK = 32 K-slab staged in LDS
// (row stride 36 floats: conflict-free ds_read_b128), double-buffered with
// register prefetch of the next slab.  Lane half h of every MFMA step s
// consumes k = 16h + s, so each lane reads its 16 k-values with 4 x
// ds_read_b128 per 32-row block.
//
// Every global access is a raw buffer op on a wave-uniform descriptor: rows
// or K columns out of range (and empty gather slots) get an offset beyond
// the descriptor's extent, so loads return 0 and stores are dropped by the
// hardware -- no per-element branches, which hipcc would otherwise turn into
// one `s_waitcnt vmcnt(0)` per load and serialise the prefetch.
#pragma once
#include <climits>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "gemm_common.h"


namespace {

using namespace sfxg;


// Persistent tile loop: each workgroup walks output tiles blockIdx.x, +gridDim.x, ... and prefetches
// the first K-slab of its NEXT tile while it computes the last slab and runs the epilogue of the
// current one, so the global-load latency of a tile start and the epilogue stores overlap (short-K
// GEMMs -- K = 64..256 on most PTv3 layers -- are otherwise latency-bound).
// MODE: how the A rows of a tile are found (compile-time so the load path has no runtime branches)

// SPLIT: the fp32 operands are split into three bf16 terms on the LDS store and every 32x32x16 block
// product is formed from the six leading term products (t0t0, t0t1, t1t0, t0t2, t1t1, t2t0; the dropped
// ones are <= 2^-24 relative) on v_mfma_f32_32x32x16_bf16 with fp32 accumulation: fp32 accuracy at
// 6 x 32 cycles per 32x32x16 block against 8 x 64 for v_mfma_f32_32x32x2_f32.  The split image is 1.5x
// the fp32 one, so LDS is single-buffered (register prefetch of the next slab, two barriers per slab).
//
// NW = waves per workgroup: 4 (2 workgroups per CU) or 8 (one 512-thread workgroup per CU, the large
// split tiles: 256x128 / 128x256 at 64x64 per wave, LDS double-buffered).
// Split LDS image: per buffer and term a [rows][32] bf16 array with 64-byte rows and no padding; the
// 16-byte chunk c of row r sits at chunk c ^ ((r >> 2) & 3), which makes the fragment reads (16 rows x one
// chunk per quarter-wave) and the staging writes (4 rows x 64 B per half-wave) bank-conflict free.
//
// SPL = 2 (the default for K >= 64): fp16x2 -- every operand row is scaled by its own power of two and split
// into two fp16 terms (split2h); a block is h*h + h*l + l*h on v_mfma_f32_32x32x16_f16 (three products, two
// LDS term images).  W arrives pre-split (sfx_weight_split: per-row scale, 1/s per output column applied in the
// epilogue).  A' rows are scaled online by the staging threads: a row's first non-zero slab puts its maximum in
// [2^12, 2^13); a later slab that would leave the fp16 range (|x s| > 65504) lowers the row's scale, and the
// staging waves post the factor (a power of two) with the slab (s_fac, any-change flag s_flag) so the compute
// waves rescale that row's accumulators before adding it.  The epilogue unscales each row by its final 1/s.
// Error: that of fp32 arithmetic (dropped l*l <= 2^-22 relative, products exact in fp32) for every row,
// whatever the other rows' magnitudes.
template <int BM, int BN, int WGM, int NW, bool VEC, int MODE, int SPL>
__global__ void __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) gemm_kernel(GemmArgs p, int tiles_n, int total_tiles) {
  constexpr bool SPLIT = SPL != 0;
  constexpr bool F16 = SPL == 2 || SPL == 1;   // fp16 terms (SPL 1: the leading term only)
  constexpr int NTERM = SPL == 1 ? 1 : (F16 ? 2 : 3);  // LDS term images per operand
  static_assert(SPL == 0 || SPL == 1 || SPL == 2 || SPL == 3, "operand precision");
  constexpr int NT = NW * 64;                  // threads
  constexpr int WGN = NW / WGM;                // waves along N
  constexpr int WM = BM / WGM, WN = BN / WGN;  // wave sub-tile
  constexpr int MB = WM / 32, NB = WN / 32;    // 32x32 MFMA blocks per wave
  constexpr int RPP = NT / 8;                  // staging rows per pass (8 threads x 4 floats per row)
  static_assert(WM % 32 == 0 && WN % 32 == 0 && (BM * BK / 4) % NT == 0 && (BN * BK / 4) % NT == 0,
                "tile shape must split into 32x32 MFMA blocks and whole staging passes");
  static_assert(SPLIT || NW == 4, "fp32 tiles run 4 waves");
  constexpr int A_ITERS = BM * BK / 4 / NT;
  constexpr int W_ITERS = BN * BK / 4 / NT;
  constexpr int NBUF = SPLIT ? (NW == 8 ? SFX_NBUF8 : 1) : 2;
  // fp32: double-buffered [row][k] images (row stride 36); SPLIT: NBUF x 3 swizzled bf16 term images
  // (fp16x2 appends the per-row scale state: [NBUF][BM] factors, [2][BM] 1/s by segment parity, [NBUF] flags --
  // in the same LDS object: a further __shared__ object can make hipcc wait vmcnt(0) before ds_reads)
  constexpr int AUX_FLOATS = F16 ? NBUF * BM + 2 * BM + 4 : 0;
  constexpr int A_FLOATS = (SPLIT ? NBUF * NTERM * BM * BK / 2 : 2 * BM * LDS_STRIDE) + AUX_FLOATS;
  constexpr int W_FLOATS = SPLIT ? NBUF * NTERM * BN * BK / 2 : 2 * BN * LDS_STRIDE;
  __shared__ __attribute__((aligned(16))) float sAraw[A_FLOATS];
  __shared__ __attribute__((aligned(16))) float sWraw[W_FLOATS];
  float (*sA)[BM * LDS_STRIDE] = reinterpret_cast<float (*)[BM * LDS_STRIDE]>(sAraw);
  float (*sW)[BN * LDS_STRIDE] = reinterpret_cast<float (*)[BN * LDS_STRIDE]>(sWraw);
  char* sAs = reinterpret_cast<char*>(sAraw);  // [NBUF][NTERM][BM][64 B]
  char* sWs = reinterpret_cast<char*>(sWraw);  // [NBUF][NTERM][BN][64 B]
  // byte offset of the 4-element group at k = c4 * 4 (c4 = 0..7) of row r in a swizzled term image
  auto swz = [](int r, int c4) -> int { return r * 64 + ((((c4 >> 1) ^ (r >> 2)) & 3) << 4) + ((c4 & 1) << 3); };
  float* s_fac = sAraw + (A_FLOATS - AUX_FLOATS);   // [NBUF][BM]
  float* s_inv = s_fac + NBUF * BM;                  // [2][BM]: a segment's epilogue reads its own copy while the
                                                     // next segment's first slab is staged into the other
  int* s_flag = reinterpret_cast<int*>(s_inv + 2 * BM);  // [NBUF]

  const int g = blockIdx.z;
  const float* A = p.A + g * p.gA;
  const float* bias = p.bias ? p.bias + g * p.gB : nullptr;
  float* Y = p.Y + g * p.gY;
  const __amdgpu_buffer_rsrc_t rA = rsrc(A);
  const __amdgpu_buffer_rsrc_t rY = rsrc(Y);
  const __amdgpu_buffer_rsrc_t rR = rsrc(p.R ? p.R : Y);
  const __amdgpu_buffer_rsrc_t rP = rsrc(p.Ypre ? p.Ypre : Y);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int h = lane >> 5, l32 = lane & 31;
  const int K = p.K;
  const int nk = (K + BK - 1) / BK;
  if constexpr (F16) {
    if (tid < NBUF) s_flag[tid] = 0;  // (published by the first barrier)
  }
  // byte offsets fit 31 bits (host checks every operand against the 2 GiB buffer range)
  const unsigned lda32 = (unsigned)p.lda, ldw32 = (unsigned)p.ldw, ldy32 = (unsigned)p.ldy, ldws32 = (unsigned)p.ldws;
  const unsigned ldr32 = (unsigned)p.ldr, ldp32 = (unsigned)p.ldypre;
  const int lrow = tid >> 3, lcol = (tid & 7) * 4;  // staging coordinates: rows lrow + RPP i, cols lcol..+3

  // per-tile geometry (all wave-uniform)
  struct Tile {
    int m0, n0, M;
    const int* gidx;
    int gstride;
    const int* out_rows;
    const float* W;       // W, or its pre-split image (SPL == 2)
    const float* winv;    // 1/s per W row (SPL == 2)
  };
  auto tile_info = [&](int t) -> Tile {
    Tile ti;
    const int tm = t / tiles_n, tn = t - tm * tiles_n;
    ti.n0 = tn * BN;
    ti.m0 = tm * BM;
    ti.M = p.M;
    ti.gidx = MODE == MODE_DENSE ? nullptr : p.gidx;
    ti.gstride = p.gstride;
    ti.out_rows = p.out_rows;
    ti.W = (F16 ? p.Wsp : p.W) + g * p.gW;
    ti.winv = p.winv ? p.winv + g * p.gWinv : nullptr;
    if constexpr (MODE == MODE_PAIR) {
      int sl = 0;
      for (int q = 1; q < p.num_slices; ++q)
        if (p.slice_tile_off[q] <= tm) sl = q;
      const int base = p.slice_pair_off[sl];
      ti.M = p.slice_pair_off[sl + 1] - base;
      ti.m0 = (tm - p.slice_tile_off[sl]) * BM;
      ti.gidx = p.pair_in + base;
      ti.gstride = 1;
      ti.out_rows = p.pair_out + base;
      ti.W = (F16 ? p.Wsp : p.W) + sl * p.slice_w_stride;
      if (p.winv) ti.winv = p.winv + sl * p.slice_winv_stride;
    }
    return ti;
  };

  // Gathered A rows: with one segment (S == 1, every gathered GEMM the model runs) the row index of a
  // staging row is the same for all K-slabs of a tile, so it is fetched once per tile -- one tile ahead,
  // together with the previous tile's work -- and the slab loads never wait on an index load.
  // With S > 1 the index depends on the slab and is re-fetched per slab.
  int grow[A_ITERS];
  auto load_rows = [&](const Tile& ti, int kt, int (&rows)[A_ITERS]) {
    if constexpr (MODE != MODE_DENSE) {
      const __amdgpu_buffer_rsrc_t rG = rsrc(ti.gidx);
      const int seg = MODE == MODE_GATHERS ? (kt * BK + lcol) / p.Kseg : 0;
#pragma unroll
      for (int i = 0; i < A_ITERS; ++i) {
        const int m = ti.m0 + lrow + RPP * i;
        rows[i] = bload1i(rG, (m < ti.M && seg < p.S) ? ((unsigned)m * (unsigned)ti.gstride + (unsigned)seg) * 4u
                                                      : OOB);
      }
    }
  };

  float4 ra[A_ITERS], rw[W_ITERS];
  auto load_tiles = [&](const Tile& ti, int kt, bool first) {
    const __amdgpu_buffer_rsrc_t rW = rsrc(ti.W);
    const int k = kt * BK + lcol;
    const bool kin = k < K && !(p.dbg & 2);
    int seg = 0, kk = k;
    if constexpr (MODE == MODE_GATHERS) {
      seg = k / p.Kseg;
      kk = k - seg * p.Kseg;
    }
#pragma unroll
    for (int i = 0; i < A_ITERS; ++i) {
      const int m = ti.m0 + lrow + RPP * i;
      const bool mok = m < ti.M;
      unsigned off;
      if constexpr (MODE != MODE_DENSE) {
        const int r = grow[i];
        off = (mok && r >= 0 && kin && seg < p.S) ? ((unsigned)r * lda32 + (unsigned)kk) * 4u : OOB;
      } else {
        off = (mok && kin) ? ((unsigned)m * lda32 + (unsigned)kk) * 4u : OOB;
      }
      if (VEC) {
        ra[i] = bload4(rA, off);
      } else {
        float4 v;
        v.x = bload1(rA, (k + 0 < K) ? off : OOB);
        v.y = bload1(rA, (k + 1 < K) ? off + 4 : OOB);
        v.z = bload1(rA, (k + 2 < K) ? off + 8 : OOB);
        v.w = bload1(rA, (k + 3 < K) ? off + 12 : OOB);
        ra[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < W_ITERS; ++i) {
      const int n = ti.n0 + lrow + RPP * i;
      const unsigned off = (n < p.N && kin) ? ((unsigned)n * (F16 ? ldws32 : ldw32) + (unsigned)k) * 4u : OOB;
      if (VEC) {
        rw[i] = bload4(rW, off);
      } else {
        float4 v;
        v.x = bload1(rW, (k + 0 < K) ? off : OOB);
        v.y = bload1(rW, (k + 1 < K) ? off + 4 : OOB);
        v.z = bload1(rW, (k + 2 < K) ? off + 8 : OOB);
        v.w = bload1(rW, (k + 3 < K) ? off + 12 : OOB);
        rw[i] = v;
      }
    }
  };
  // SPL == 2 per-row scale state of the staged rows lrow + RPP i (exponent, scale, overflow threshold) and the
  // stamp of the last stored slab (the flag that asks the compute waves to rescale carries it)
  int erow[A_ITERS];
  float srow[A_ITERS], thr[A_ITERS];
#pragma unroll
  for (int i = 0; i < A_ITERS; ++i) { erow[i] = INT_MIN; srow[i] = 1.f; thr[i] = 0.f; }
  int sq = 0, cq = 0;
  int sp = 0;  // segment parity (the s_inv copy of the current segment)
  // par: parity of the segment whose rows are staged (selects its s_inv copy)
  auto store_tiles = [&](int buf, bool first, int par) {
    if (p.dbg & 8) return;
    if constexpr (SPLIT) {
      const int b = NBUF == 2 ? buf : 0;
      if constexpr (F16) {
        ++sq;
        float m[A_ITERS];
        bool over = false;
#pragma unroll
        for (int i = 0; i < A_ITERS; ++i) {
          m[i] = fmaxf(fmaxf(fabsf(ra[i].x), fabsf(ra[i].y)), fmaxf(fabsf(ra[i].z), fabsf(ra[i].w)));
          over |= m[i] > thr[i];
        }
        bool dec = false;
        if (first || __builtin_amdgcn_ballot_w64(over) != 0) {
          // slow path (a segment's first slab, a row's first non-zero slab, or a slab that would overflow fp16):
          // row maxima over the row's 8 staging lanes, new exponents, rescale factors and 1/s
#pragma unroll
          for (int i = 0; i < A_ITERS; ++i) {
            float mr = m[i];
            mr = fmaxf(mr, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mr), 0xB1, 0xF, 0xF, false)));
            mr = fmaxf(mr, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mr), 0x4E, 0xF, 0xF, false)));
            mr = fmaxf(mr, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mr), 0x141, 0xF, 0xF, false)));
            int e = first ? INT_MIN : erow[i];
            float fac = 1.f;
            bool chg = first;
            if (mr > 0.f && mr <= 3.4028235e38f) {
              int e2 = 13 - __builtin_amdgcn_frexp_expf(mr);  // row max in [2^12, 2^13)
              e2 = e2 > 126 ? 126 : (e2 < -126 ? -126 : e2);
              if (e == INT_MIN) {  // the row's accumulators are still zero: no rescale
                e = e2;
                chg = true;
              } else if (mr * srow[i] > 65504.f) {
                fac = ldexpf(1.f, e2 - e);
                e = e2;
                chg = true;
                dec = true;
              }
            }
            erow[i] = e;
            const bool set = e != INT_MIN;
            srow[i] = set ? ldexpf(1.f, e) : 1.f;
            thr[i] = set ? ldexpf(65504.f, -e) : 0.f;
            if ((tid & 7) == 0) {
              s_fac[b * BM + lrow + RPP * i] = fac;
              if (chg) s_inv[par * BM + lrow + RPP * i] = set ? ldexpf(1.f, -e) : 1.f;
            }
          }
        } else if ((tid & 7) == 0) {
#pragma unroll
          for (int i = 0; i < A_ITERS; ++i) s_fac[b * BM + lrow + RPP * i] = 1.f;
        }
        if (__builtin_amdgcn_ballot_w64(dec) != 0 && lane == 0) s_flag[b] = sq;
#pragma unroll
        for (int i = 0; i < A_ITERS; ++i) {
          uint2 t[2];
          split2h(ra[i], srow[i], t);
          const int o = swz(lrow + RPP * i, lcol >> 2);
          *reinterpret_cast<uint2*>(sAs + ((b * NTERM + 0) * BM) * 64 + o) = t[0];
          if constexpr (NTERM == 2) *reinterpret_cast<uint2*>(sAs + ((b * NTERM + 1) * BM) * 64 + o) = t[1];
        }
#pragma unroll
        for (int i = 0; i < W_ITERS; ++i) {  // pre-split: h terms in .x/.y, l terms in .z/.w
          const uint4 w = __builtin_bit_cast(uint4, rw[i]);
          const int o = swz(lrow + RPP * i, lcol >> 2);
          *reinterpret_cast<uint2*>(sWs + ((b * NTERM + 0) * BN) * 64 + o) = make_uint2(w.x, w.y);
          if constexpr (NTERM == 2) *reinterpret_cast<uint2*>(sWs + ((b * NTERM + 1) * BN) * 64 + o) = make_uint2(w.z, w.w);
        }
        return;
      } else {
#pragma unroll
      for (int i = 0; i < A_ITERS; ++i) {
        uint2 t[NTERM];
        split3(ra[i], t);
        const int o = swz(lrow + RPP * i, lcol >> 2);
#pragma unroll
        for (int q = 0; q < NTERM; ++q) *reinterpret_cast<uint2*>(sAs + ((b * NTERM + q) * BM) * 64 + o) = t[q];
      }
#pragma unroll
      for (int i = 0; i < W_ITERS; ++i) {
        uint2 t[NTERM];
        split3(rw[i], t);
        const int o = swz(lrow + RPP * i, lcol >> 2);
#pragma unroll
        for (int q = 0; q < NTERM; ++q) *reinterpret_cast<uint2*>(sWs + ((b * NTERM + q) * BN) * 64 + o) = t[q];
      }
      return;
      }
    }
#pragma unroll
    for (int i = 0; i < A_ITERS; ++i)
      *reinterpret_cast<float4*>(&sA[buf][(lrow + RPP * i) * LDS_STRIDE + lcol]) = ra[i];
#pragma unroll
    for (int i = 0; i < W_ITERS; ++i)
      *reinterpret_cast<float4*>(&sW[buf][(lrow + RPP * i) * LDS_STRIDE + lcol]) = rw[i];
  };

  floatx16 acc[MB][NB];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  };

  // Epilogue operands of the current tile (bias/scale/shift per column, output row per accumulator row)
  // are fetched BEFORE the next tile's prefetch is issued, so the epilogue never waits on the prefetch.
  float ebias[NB], escale[NB], eshift[NB], ewinv[NB];
  int mrow[MB][16];
  float ymax = 0.f;  // running max |Y| of this workgroup's outputs (p.y_amax)
  auto load_mrow = [&](const Tile& ti, __amdgpu_buffer_rsrc_t rO) {
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mt = ti.m0 + wm * WM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        mrow[a][r] = bload1i(rO, mt < ti.M ? (unsigned)mt * 4u : OOB);
      }
  };
  auto pre_epilogue = [&](const Tile& ti) {
    // branch-free: absent operands read through an out-of-range offset (-> 0) and are then selected away
    const __amdgpu_buffer_rsrc_t rB = rsrc(bias ? bias : p.W);
    const __amdgpu_buffer_rsrc_t rS = rsrc(p.scale ? p.scale : p.W);
    const __amdgpu_buffer_rsrc_t rH = rsrc(p.shift ? p.shift : p.W);
    const __amdgpu_buffer_rsrc_t rO = rsrc(ti.out_rows ? (const void*)ti.out_rows : (const void*)p.W);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int n = ti.n0 + wn * WN + b * 32 + l32;
      const unsigned off = n < p.N ? (unsigned)n * 4u : OOB;
      const float bv = bload1(rB, bias ? off : OOB);
      const float sv = bload1(rS, p.scale ? off : OOB);
      const float hv = bload1(rH, p.shift ? off : OOB);
      ebias[b] = bv;
      escale[b] = sv;  // raw loads; the defaults for absent operands are selected in the epilogue, so
      eshift[b] = hv;  // nothing here waits on them
      if constexpr (F16) ewinv[b] = bload1(rsrc(ti.winv), off);
    }
    // output-row remaps (pair mode's pair_out; an out_rows argument of the other modes) are loaded in the
    // epilogue, keeping 16 * MB registers free across the MFMAs
    (void)rO;
  };
  // output row of accumulator row r of block a (-1: outside the tile)
  auto resolve_rows = [&](const Tile& ti) {
    const bool remap = ti.out_rows != nullptr;
    if constexpr (MODE != MODE_PAIR) {
      if (remap) load_mrow(ti, rsrc(ti.out_rows));
    }
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mt = ti.m0 + wm * WM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        mrow[a][r] = mt < ti.M ? (remap ? mrow[a][r] : mt) : -1;
      }
#pragma unroll
    for (int b = 0; b < NB; ++b) escale[b] = p.scale ? escale[b] : 1.f;
  };

  // epilogue: branch-free buffer stores (row -1 / out-of-range column -> dropped); the runtime epilogue
  // options are tested once per 16-element column strip, never per element.
  // Direct-row epilogue (no output-row remap, the common case): every operand row r of a 32-row block is
  // base + rowc(r) * ld with a wave-uniform rowc(r) * ld, so an address costs one add; rows past M fall
  // outside the descriptor extent (M * ld * 4 bytes) and columns past N get a base past every extent, so
  // the hardware drops / zero-fills them with no per-element selects.  One FMA applies bias/scale/shift.
  constexpr unsigned OOBX = 0x80000000u;
  auto rowc = [](int r) -> unsigned { return (unsigned)((r & 3) + 8 * (r >> 2)); };
  auto direct_epilogue = [&](const Tile& ti, bool partial, bool owner0) {
    const unsigned Mu = (unsigned)ti.M;
    const __amdgpu_buffer_rsrc_t rYd = rsrc_ext(Y, Mu * ldy32 * 4u);
    const __amdgpu_buffer_rsrc_t rPd = rsrc_ext(p.Ypre ? p.Ypre : Y, Mu * ldp32 * 4u);
    const __amdgpu_buffer_rsrc_t rRd = rsrc_ext(p.R ? p.R : Y, p.ridx ? OOB : Mu * ldr32 * 4u);
    const __amdgpu_buffer_rsrc_t rSd = rsrc_ext(p.rowscale ? p.rowscale : p.W, Mu * 4u);
    const unsigned ldd32 = (unsigned)p.ld_dact;
    const __amdgpu_buffer_rsrc_t rDd = rsrc_ext(p.dact_pre ? p.dact_pre : p.W, Mu * ldd32 * 4u);
    const __amdgpu_buffer_rsrc_t rI = rsrc(p.ridx ? (const void*)p.ridx : (const void*)p.W);
#pragma unroll
    for (int a = 0; a < MB; ++a) {
      const unsigned mb = (unsigned)(ti.m0 + wm * WM + a * 32 + 4 * h);  // row of r = 0 (this lane half)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int n = ti.n0 + wn * WN + b * 32 + l32;
        const bool nok = n < p.N;
        const bool do_act = n < p.act_ncols;
        const unsigned by = nok ? (mb * ldy32 + (unsigned)n) * 4u : OOBX;
        const float c1 = p.scale ? escale[b] : 1.f;
        const float cb = ebias[b] * c1 + eshift[b];
        const float c0 = (partial && !owner0) ? 0.f : cb;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = __builtin_fmaf(acc[a][b][r], c1, c0);
        if (p.Ypre && p.pre_before_act) {
          const unsigned bp = nok ? (mb * ldp32 + (unsigned)n) * 4u : OOBX;
#pragma unroll
          for (int r = 0; r < 16; ++r) bstore1(rPd, bp + rowc(r) * ldp32 * 4u, v[r]);
        }
        if (p.act == ACT_GELU) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? gelu_erf(v[r]) : v[r];
        } else if (p.act == ACT_RELU) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? fmaxf(v[r], 0.f) : v[r];
        } else if (p.act == ACT_TANH) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? tanhf(v[r]) : v[r];
        }
        if (p.rowscale) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] *= bload1(rSd, (mb + rowc(r)) * 4u);
        }
        if (p.dact) {
          const unsigned bd = nok ? (mb * ldd32 + (unsigned)n) * 4u : OOBX;
          float pre[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) pre[r] = bload1(rDd, bd + rowc(r) * ldd32 * 4u);
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? v[r] * dact_grad(p.dact, pre[r]) : v[r];
        }
        if (p.Ypre && !p.pre_before_act) {
          const unsigned bp = nok ? (mb * ldp32 + (unsigned)n) * 4u : OOBX;
#pragma unroll
          for (int r = 0; r < 16; ++r) bstore1(rPd, bp + rowc(r) * ldp32 * 4u, v[r]);
        }
        if (p.R && owner0) {
          float rv[16];
          if (p.ridx) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const unsigned m = mb + rowc(r);
              const int ri = bload1i(rI, m < Mu ? m * 4u : OOB);
              rv[r] = bload1(rRd, (nok && m < Mu) ? ((unsigned)ri * ldr32 + (unsigned)n) * 4u : OOB);
            }
          } else {
            const unsigned br = nok ? (mb * ldr32 + (unsigned)n) * 4u : OOBX;
#pragma unroll
            for (int r = 0; r < 16; ++r) rv[r] = bload1(rRd, br + rowc(r) * ldr32 * 4u);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] += rv[r];
        }
        if (p.y_amax) {
#pragma unroll
          for (int r = 0; r < 16; ++r) ymax = fmaxf(ymax, fabsf(v[r]));
        }
        if (partial) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v[r], rYd, by + rowc(r) * ldy32 * 4u, 0, 0);
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) bstore1(rYd, by + rowc(r) * ldy32 * 4u, v[r]);
        }
      }
    }
  };

  auto epilogue = [&](const Tile& ti, bool partial, bool owner0) {
    if (p.dbg & 4) return;
    if constexpr (F16) {  // undo the row scales of A' and W (powers of two: exact)
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const float4 f = *reinterpret_cast<const float4*>(s_inv + sp * BM + wm * WM + a * 32 + 8 * gq + 4 * h);
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            acc[a][b][4 * gq + 0] *= f.x * ewinv[b];
            acc[a][b][4 * gq + 1] *= f.y * ewinv[b];
            acc[a][b][4 * gq + 2] *= f.z * ewinv[b];
            acc[a][b][4 * gq + 3] *= f.w * ewinv[b];
          }
        }
    }
    if constexpr (MODE != MODE_PAIR) {
      if (!ti.out_rows) {
        direct_epilogue(ti, partial, owner0);
        return;
      }
    }
    if constexpr (MODE == MODE_PAIR) {
      // partial sums of one neighbour offset: accumulated into the output rows (float atomics), or, with
      // pair_store, stored as row `pair index` of a partials matrix that the consumer sums per output row in a
      // fixed offset order (sfx_cpe_residual_ln_pairs: no atomics, bitwise reproducible)
      const __amdgpu_buffer_rsrc_t rO = rsrc(ti.out_rows);
      const int pbase = (int)(ti.out_rows - p.pair_out);
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        int orow[16];
        bool ok[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mt = ti.m0 + wm * WM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          ok[r] = mt < ti.M;
          orow[r] = p.pair_store ? pbase + mt : bload1i(rO, ok[r] ? (unsigned)mt * 4u : OOB);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const int n = ti.n0 + wn * WN + b * 32 + l32;
          const bool nok = n < p.N;
          if (p.pair_store) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
              bstore1(rY, (nok && ok[r]) ? ((unsigned)orow[r] * ldy32 + (unsigned)n) * 4u : OOB, acc[a][b][r]);
            continue;
          }
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(
                acc[a][b][r], rY, (nok && ok[r]) ? ((unsigned)orow[r] * ldy32 + (unsigned)n) * 4u : OOB, 0, 0);
        }
      }
      return;
    }
    resolve_rows(ti);
#pragma unroll
    for (int a = 0; a < MB; ++a) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int n = ti.n0 + wn * WN + b * 32 + l32;
        const bool nok = n < p.N;
        const bool do_act = n < p.act_ncols;
        float v[16];
        if (partial) {  // Stream-K piece: linear epilogue split -- only the k-slab-0 owner adds bias/shift
          const float c0 = owner0 ? ebias[b] * escale[b] + eshift[b] : 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = acc[a][b][r] * escale[b] + c0;
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = (acc[a][b][r] + ebias[b]) * escale[b] + eshift[b];
        }
        if (p.Ypre && p.pre_before_act) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            bstore1(rP, (nok && m >= 0) ? ((unsigned)m * ldp32 + (unsigned)n) * 4u : OOB, v[r]);
          }
        }
        if (p.act == ACT_GELU) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? gelu_erf(v[r]) : v[r];
        } else if (p.act == ACT_RELU) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? fmaxf(v[r], 0.f) : v[r];
        } else if (p.act == ACT_TANH) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? tanhf(v[r]) : v[r];
        }
        if (p.rowscale) {
          const __amdgpu_buffer_rsrc_t rRS = rsrc(p.rowscale);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            v[r] *= bload1(rRS, m >= 0 ? (unsigned)m * 4u : OOB);
          }
        }
        if (p.dact) {
          const __amdgpu_buffer_rsrc_t rD = rsrc(p.dact_pre);
          const unsigned ldd = (unsigned)p.ld_dact;
          float pre[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            pre[r] = bload1(rD, (nok && m >= 0) ? ((unsigned)m * ldd + (unsigned)n) * 4u : OOB);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = do_act ? v[r] * dact_grad(p.dact, pre[r]) : v[r];
        }
        if (p.Ypre && !p.pre_before_act) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            bstore1(rP, (nok && m >= 0) ? ((unsigned)m * ldp32 + (unsigned)n) * 4u : OOB, v[r]);
          }
        }
        if (p.R && owner0) {
          float rv[16];
          const __amdgpu_buffer_rsrc_t rI = rsrc(p.ridx ? (const void*)p.ridx : (const void*)p.W);
          int rr[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            const int ri = bload1i(rI, (p.ridx && m >= 0) ? (unsigned)m * 4u : OOB);
            rr[r] = p.ridx ? ri : m;
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            rv[r] = bload1(rR, (nok && m >= 0) ? ((unsigned)rr[r] * ldr32 + (unsigned)n) * 4u : OOB);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] += rv[r];
        }
        if (p.y_amax) {
#pragma unroll
          for (int r = 0; r < 16; ++r) ymax = fmaxf(ymax, mrow[a][r] >= 0 ? fabsf(v[r]) : 0.f);
        }
        if (partial) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(
                v[r], rY, (nok && m >= 0) ? ((unsigned)m * ldy32 + (unsigned)n) * 4u : OOB, 0, 0);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow[a][r];
            bstore1(rY, (nok && m >= 0) ? ((unsigned)m * ldy32 + (unsigned)n) * 4u : OOB, v[r]);
          }
        }
      }
    }
  };

  // SPLIT: k16 steps [s0, s1) of the slab
  auto compute_split = [&](int buf, int s0, int s1) {
    const int bb = NBUF == 2 ? buf : 0;
    typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
    typedef typename std::conditional<F16, f16x8, bf16x8>::type frag_t;
#pragma unroll
    for (int s = s0; s < s1; ++s) {
      frag_t af[MB][NTERM], wf[NB][NTERM];
#pragma unroll
      for (int q = 0; q < NTERM; ++q) {
#pragma unroll
        for (int a = 0; a < MB; ++a) {
          const int r = wm * WM + a * 32 + l32;
          af[a][q] = __builtin_bit_cast(
              frag_t, *reinterpret_cast<const uint4*>(sAs + ((bb * NTERM + q) * BM) * 64 + swz(r, 4 * s + 2 * h)));
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const int r = wn * WN + b * 32 + l32;
          wf[b][q] = __builtin_bit_cast(
              frag_t, *reinterpret_cast<const uint4*>(sWs + ((bb * NTERM + q) * BN) * 64 + swz(r, 4 * s + 2 * h)));
        }
      }
      // smallest terms first; the (a, b) blocks interleave so consecutive MFMAs are independent
      if constexpr (F16) {
        constexpr int QA[3] = {1, 0, 0}, QW[3] = {0, 1, 0};
#pragma unroll
        for (int j = SPL == 1 ? 2 : 0; j < 3; ++j)  // SPL 1: h*h only
#pragma unroll
          for (int a = 0; a < MB; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][QA[j]], wf[b][QW[j]], acc[a][b], 0, 0, 0);
      } else {
        constexpr int QA[6] = {2, 1, 0, 1, 0, 0}, QW[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int j = 0; j < 6; ++j)
#pragma unroll
          for (int a = 0; a < MB; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][QA[j]], wf[b][QW[j]], acc[a][b], 0, 0, 0);
      }
    }
  };
  auto compute = [&](int buf) {
    if (p.dbg & 1) return;
    if constexpr (F16) {  // a later slab lowered some rows' scales: rescale their accumulators first
      ++cq;
      const int b = NBUF == 2 ? buf : 0;
      if (__builtin_amdgcn_readfirstlane(s_flag[b]) == cq) {
#pragma unroll
        for (int a = 0; a < MB; ++a)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const float4 f = *reinterpret_cast<const float4*>(s_fac + b * BM + wm * WM + a * 32 + 8 * gq + 4 * h);
#pragma unroll
            for (int bb = 0; bb < NB; ++bb) {
              acc[a][bb][4 * gq + 0] *= f.x;
              acc[a][bb][4 * gq + 1] *= f.y;
              acc[a][bb][4 * gq + 2] *= f.z;
              acc[a][bb][4 * gq + 3] *= f.w;
            }
          }
      }
    }
    if constexpr (SPLIT) {
      compute_split(buf, 0, BK / 16);
      return;
    }
    const float* a_lds = &sA[buf][(wm * WM + l32) * LDS_STRIDE + h * 16];
    const float* w_lds = &sW[buf][(wn * WN + l32) * LDS_STRIDE + h * 16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float4 af[MB], wf[NB];
#pragma unroll
      for (int a = 0; a < MB; ++a) af[a] = *reinterpret_cast<const float4*>(a_lds + a * 32 * LDS_STRIDE + 4 * c);
#pragma unroll
      for (int b = 0; b < NB; ++b) wf[b] = *reinterpret_cast<const float4*>(w_lds + b * 32 * LDS_STRIDE + 4 * c);
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].x, wf[b].x, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].y, wf[b].y, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].z, wf[b].z, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].w, wf[b].w, acc[a][b], 0, 0, 0);
        }
    }
  };

  // XCD-aware numbering: workgroups are dealt round-robin to the 8 XCDs (blockIdx % 8), so give each XCD
  // a contiguous range of logical ids -- consecutive tiles (same A row-block, tn fastest) then run on one
  // XCD and share its L2 instead of being fetched once per XCD.
  const int nwg = (int)gridDim.x;
  const int lid = (nwg % 8 == 0) ? (int)(blockIdx.x % 8) * (nwg / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  // current segment: tile t, K-slabs [kb, ke).  Persistent: whole tiles lid, lid + nwg, ...;  Stream-K: the
  // contiguous iteration range [it_begin, it_end) of tiles x slabs.
  int t, kb = 0, ke = nk;
  long long it_end = 0;
  if (p.sk) {
    const long long total_it = (long long)total_tiles * nk;
    const long long it0 = total_it * lid / nwg;
    it_end = total_it * (lid + 1) / nwg;
    if (it0 >= it_end) return;
    t = (int)(it0 / nk);
    kb = (int)(it0 - (long long)t * nk);
    ke = (int)min((long long)nk, kb + (it_end - it0));
  } else {
    t = lid;
    if (t >= total_tiles) return;
  }
  constexpr bool per_tile_rows = MODE == MODE_GATHER1 || MODE == MODE_PAIR;
  Tile ti = tile_info(t);
  load_rows(ti, kb, grow);
  load_tiles(ti, kb, true);
  store_tiles(0, true, sp);
  __syncthreads();
  int buf = 0;
  while (true) {
    int nt, nke = nk;
    bool has_next;
    if (p.sk) {
      nt = t + 1;
      has_next = (long long)nt * nk < it_end;
      if (has_next) nke = (int)min((long long)nk, it_end - (long long)nt * nk);
    } else {
      nt = t + nwg;
      has_next = nt < total_tiles;
    }
    const Tile tn = has_next ? tile_info(nt) : ti;
    int grow_next[A_ITERS];
    if constexpr (per_tile_rows) load_rows(tn, 0, grow_next);  // next tile's gather rows, a whole tile ahead
    zero_acc();
    for (int kt = kb; kt + 1 < ke; ++kt) {
      if constexpr (MODE == MODE_GATHERS) load_rows(ti, kt + 1, grow);
      load_tiles(ti, kt + 1, false);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the MFMAs it overlaps
      compute(buf);
      // ... and the staging of the prefetched slab behind them: hipcc otherwise hoists the fp16x2 row-maximum VALU
      // of store_tiles between the MFMAs, with vmcnt waits that stall the wave while the matrix pipe idles
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NBUF == 1) __syncthreads();  // single LDS buffer: every wave is done reading it
      store_tiles(buf ^ 1, false, sp);
      __syncthreads();
      if constexpr (NBUF == 2) buf ^= 1;
    }
    // last slab of the segment: its epilogue operands, then the first slab of the next segment in flight
    // while the last MFMAs and the epilogue run
    pre_epilogue(ti);
    if (has_next) {
      if constexpr (per_tile_rows) {
#pragma unroll
        for (int i = 0; i < A_ITERS; ++i) grow[i] = grow_next[i];
      } else {
        load_rows(tn, 0, grow);
      }
      load_tiles(tn, 0, true);
    }
    __builtin_amdgcn_sched_barrier(0);
    compute(buf);
    __builtin_amdgcn_sched_barrier(0);
    epilogue(ti, kb != 0 || ke != nk, kb == 0);
    if (!has_next) break;
    if constexpr (NBUF == 1) __syncthreads();
    __builtin_amdgcn_sched_barrier(0);  // the next tile's staging (and its load waits) after the epilogue stores
    store_tiles(buf ^ 1, true, sp ^ 1);
    __syncthreads();
    if constexpr (NBUF == 2) buf ^= 1;
    sp ^= 1;
    t = nt;
    ti = tn;
    kb = 0;
    ke = nke;
  }
  if (p.y_amax) {
    __shared__ float ywaves[NW];
    sfx::publish_amax(ymax, p.y_amax, p.y_tag, ywaves);
  }
}
template <int BM, int BN, int WGM, int NW, int MODE>
void launch(GemmArgs a, int groups, bool vec, hipStream_t st) {
  const bool split = a.split != 0;
  const int tiles_m = tiles_m_of(a, BM);
  const int tiles_n = (int)sfx::ceil_div(a.N, BN);
  const int total = tiles_m * tiles_n;
  // persistent grid: 2 four-wave or 1 eight-wave workgroup per CU (LDS/VGPR bound), balanced so every
  // workgroup gets the same number of tiles (+-1)
  const int per_cu = NW == 4 ? kPerCu4 : kPerCu8;
  const int slots = per_cu * num_cus() / groups > 0 ? per_cu * num_cus() / groups : 1;
  int grid_x;
  if (a.sk) {
    const long long iters = (long long)total * sfx::ceil_div(a.K, BK);
    grid_x = (int)(iters < slots ? iters : slots);
    if (grid_x >= 8) grid_x = grid_x / 8 * 8;
    if (grid_x < 1) grid_x = 1;
    if (!a.pair_mode)  // partial tiles accumulate atomically: zero the N output columns first
      (void)hipMemset2DAsync(a.Y, (size_t)a.ldy * 4, 0, (size_t)a.N * 4, (size_t)a.M, st);
  } else {
    const int per = (total + slots - 1) / slots;
    grid_x = total > 0 ? (total + per - 1) / per : 1;
    if (grid_x >= 8) grid_x = (grid_x + 7) / 8 * 8;  // whole XCD groups for the XCD-aware numbering
  }
  dim3 grid(grid_x, 1, groups);
  if constexpr (NW == 8) {  // split-only tiles (vec operands)
    if (a.split == 2)
      gemm_kernel<BM, BN, WGM, 8, true, MODE, 2><<<grid, 512, 0, st>>>(a, tiles_n, total);
    else if (a.split == 1)
      gemm_kernel<BM, BN, WGM, 8, true, MODE, 1><<<grid, 512, 0, st>>>(a, tiles_n, total);
    else
      gemm_kernel<BM, BN, WGM, 8, true, MODE, 3><<<grid, 512, 0, st>>>(a, tiles_n, total);
  } else {
    if (vec && a.split == 2)
      gemm_kernel<BM, BN, WGM, 4, true, MODE, 2><<<grid, 256, 0, st>>>(a, tiles_n, total);
    else if (vec && a.split == 1)
      gemm_kernel<BM, BN, WGM, 4, true, MODE, 1><<<grid, 256, 0, st>>>(a, tiles_n, total);
    else if (vec && split)
      gemm_kernel<BM, BN, WGM, 4, true, MODE, 3><<<grid, 256, 0, st>>>(a, tiles_n, total);
    else if (vec)
      gemm_kernel<BM, BN, WGM, 4, true, MODE, 0><<<grid, 256, 0, st>>>(a, tiles_n, total);
    else
      gemm_kernel<BM, BN, WGM, 4, false, MODE, 0><<<grid, 256, 0, st>>>(a, tiles_n, total);
  }
}

}  // namespace
