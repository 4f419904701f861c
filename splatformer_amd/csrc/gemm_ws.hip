// Warp-specialised fp32-accurate GEMM for gfx950 (fp16x2 terms, per-row operand scales).
//
//   Y[m, n] = act( (sum_k A'[m, k] W[n, k] + bias[n]) * scale[n] + shift[n] ) + R[r(m), n]   (gemm_common.h)
//
// One 512-thread workgroup per CU, two roles:
//  * 4 producer waves stream K-slabs (BK = 32) of the A' and W tiles from global memory into registers two
//    slabs ahead, split every fp32 element into two fp16 terms (x*s = h + l, split2h) and store the term images
//    into a ring of NS LDS stages;
//  * 4 consumer waves (one per SIMD, next to one producer wave) hold the accumulators and issue the
//    v_mfma_f32_32x32x16_f16 products h*h + h*l + l*h of every 32x32x16 block back to back.
// One s_barrier per slab hands stage q to the consumers while the producers fill stage q+1, so the global-load
// latency, the split VALU and the LDS stores of the producers co-execute with the consumers' MFMAs on every
// SIMD instead of alternating with them (the general kernel in gemm.hip runs all waves through both phases).
// Workgroups are persistent over tiles and the slab sequence runs across tile boundaries: the producers fill
// the next tile's first slabs while the consumers run the current tile's last MFMAs and epilogue.
//
// Operand scales.  W uses one power of two per tensor (its maximum: a cached amax slot).  A' rows get their own
// power of two, chosen online by the producers: the first non-zero slab of a row puts the row's maximum in
// [2^12, 2^13); a later slab whose maximum would reach the fp16 range (|x*s| > 65504) lowers the row's scale to
// that slab's maximum and the producers post, with the slab, the factor (a power of two) by which the
// consumers rescale that row's accumulators before adding the slab (a per-stage flag says whether any row of
// the slab changed).  The epilogue unscales every accumulator row by its row's final 1/s and the tensor's
// 1/s_W -- all powers of two, so exact.  Every row therefore keeps 22 significant bits down to 2^-15 of its
// own maximum, whatever the other rows' magnitudes (rows may span the whole fp32 range).
#include <climits>
#include <type_traits>
#include <cstdlib>
#include <cstring>

#include "gemm_common.h"

namespace {

using namespace sfxg;

constexpr int WS_CONS = 4;         // consumer waves
constexpr int WS_THREADS = 512;    // 4 consumer + 4 producer waves
constexpr int E_UNSET = INT_MIN;   // row exponent before the row's first non-zero slab
#ifndef SFX_WS_TRACE
#define SFX_WS_TRACE 0  // profiling builds only: per-phase cycle sums of one producer and one consumer wave
#endif
#if SFX_WS_TRACE
__device__ unsigned long long g_ws_trace[16];
#define WS_T(v) unsigned long long v = __builtin_readcyclecounter()
#else
#define WS_T(v)
#endif
#ifndef SFX_WS_ABLATE
#define SFX_WS_ABLATE 0  // profiling builds only: 1 consumers skip the MFMAs, 2 producers skip the global loads
#endif

// f(integral_constant<int, i>) for i = 0 .. N-1: compile-time accumulator indices however large the body
// (a `#pragma unroll` loop over a large epilogue body is left rolled, which demotes the accumulators to scratch)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

struct TileGeo {
  int m0, n0, M;
  const int* gidx;
  int gstride;
  const int* out_rows;
  const float* Wsp;   // pre-split W of the tile (group / slice applied)
  const float* winv;  // its row inverse scales (or null)
};

template <int BM, int BN, int MODE>
__device__ __forceinline__ TileGeo tile_geo(const GemmArgs& p, int g, int t, int tiles_n) {
  TileGeo ti;
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  ti.n0 = tn * BN;
  ti.m0 = tm * BM;
  ti.M = p.M;
  ti.gidx = MODE == MODE_DENSE ? nullptr : p.gidx;
  ti.gstride = p.gstride;
  ti.out_rows = p.out_rows;
  ti.Wsp = p.Wsp + g * p.gW;
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
    ti.Wsp = p.Wsp + sl * p.slice_w_stride;
    if (p.winv) ti.winv = p.winv + sl * p.slice_winv_stride;
  }
  return ti;
}

// max over the 8 lanes of an aligned lane group (the 8 producer lanes that stage one row)
__device__ __forceinline__ float max8(float m) {
  m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0xB1, 0xF, 0xF, false)));   // quad [1,0,3,2]
  m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x4E, 0xF, 0xF, false)));   // quad [2,3,0,1]
  m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x141, 0xF, 0xF, false)));  // half-row mirror
  return m;
}

// (row_exp: the row exponent, gemm_common.h)

// LDS map (one __shared__ array: a second LDS object can make hipcc wait vmcnt(0) before ds_reads):
//   [NS] stages of { A terms h, l: [BM][64 B] swizzled; W terms h, l: [BN][64 B] }
//   [BM][BN + 4] float epilogue staging (a finished tile's pre-activation values)
//   [NS][BM] float row rescale factors, [2][BM] float row 1/s (by tile parity), [NS][4] int flags (one per
//   producer wave), [8] float wave maxima
template <int BM, int BN, int NS>
struct WsLds {
  static constexpr int TA = BM * 64, TW = BN * 64;
  static constexpr int STAGE = 2 * TA + 2 * TW;
  static constexpr int SLD = BN + 4;  // staging row stride (floats)
  static constexpr int STG = NS * STAGE;
  static constexpr int FAC = STG + BM * SLD * 4;
  static constexpr int INV = FAC + NS * BM * 4;
  static constexpr int FLAG = INV + 2 * BM * 4;
  static constexpr int YW = FLAG + NS * 16;
  static constexpr int BYTES = YW + 8 * 4;
  static_assert(BYTES <= 160 * 1024, "LDS budget");
};

template <int BM, int BN, int WGM, int MODE, int NS, int NSET>
__global__ void __launch_bounds__(WS_THREADS, 1) gemm_ws_kernel(GemmArgs p, int tiles_n, int total_tiles) {
  constexpr int WGN = WS_CONS / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MB = WM / 32, NB = WN / 32;
  constexpr int A_IT = BM / 32, W_IT = BN / 32;  // staged 16-byte groups per producer thread and slab
  constexpr int EPI_ITEMS = BM * BN / 4 / 256;   // staged float4 per producer thread and tile
  using L = WsLds<BM, BN, NS>;
  static_assert(WM % 32 == 0 && WN % 32 == 0 && NS >= 2 && NS <= 8 && BN % 4 == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
  float* s_stg = reinterpret_cast<float*>(smem + L::STG);
  float* s_fac = reinterpret_cast<float*>(smem + L::FAC);
  float* s_inv = reinterpret_cast<float*>(smem + L::INV);
  int* s_flag = reinterpret_cast<int*>(smem + L::FLAG);
  auto swz = [](int r, int c4) -> int { return r * 64 + ((((c4 >> 1) ^ (r >> 2)) & 3) << 4) + ((c4 & 1) << 3); };

  const int g = blockIdx.z;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int K = p.K;
  const int nk = (K + BK - 1) / BK;
  // XCD-aware, bijective numbering: consecutive logical ids (same A row-block, tn fastest) share an XCD's L2
  const int nwg = (int)gridDim.x;
  int lid;
  {
    const int xcd = (int)blockIdx.x % 8, q8 = nwg / 8, r8 = nwg % 8;
    lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (int)blockIdx.x / 8;
  }
  const int my_tiles = lid < total_tiles ? (total_tiles - lid + nwg - 1) / nwg : 0;
  const int total_q = my_tiles * nk;
  const int total_qp = (total_q + NSET - 1) / NSET * NSET;  // barrier rounds of both roles (see the producer loop)
  if (tid < NS * 4) s_flag[tid] = 0;
  float ymax = 0.f;

  if (wid >= WS_CONS) {
    // ------------------------------------------------------------------ producers
    const int pw = wid - WS_CONS;                  // producer wave: stages rows 8 pw .. 8 pw + 7 (mod 32)
    const int pt = tid - WS_CONS * 64;
    const int prow = pt >> 3, pc4 = pt & 7, pcol = pc4 * 4;
    const int lds_off = swz(prow, pc4);            // + 2048 r for row prow + 32 r (the swizzle term repeats)
    const __amdgpu_buffer_rsrc_t rA = rsrc(p.A + g * p.gA);
    const unsigned lda32 = (unsigned)p.lda, ldw32 = (unsigned)p.ldws;
    float4 ra[NSET][A_IT];
    uint4 rw[NSET][W_IT];
    int rows_cur[A_IT];  // gather rows of the slab issued next
    unsigned abase[A_IT], wbase[W_IT];  // byte offsets of the staged rows of the tile being issued (or OOB)
    // issue side: slab (iss_i, iss_kt) of tile ti_iss; ti_fol = the tile after it
    int iss_i = 0, iss_kt = 0;
    TileGeo ti_iss = tile_geo<BM, BN, MODE>(p, g, lid, tiles_n);
    TileGeo ti_fol = tile_geo<BM, BN, MODE>(p, g, lid + nwg, tiles_n);
    auto load_rows = [&](const TileGeo& ti, bool valid, int (&rows)[A_IT]) {
      const __amdgpu_buffer_rsrc_t rG = rsrc(ti.gidx);
#pragma unroll
      for (int r = 0; r < A_IT; ++r) {
        const int m = ti.m0 + prow + 32 * r;
        rows[r] = bload1i(rG, (valid && m < ti.M) ? (unsigned)m * (unsigned)ti.gstride * 4u : OOB);
      }
    };
    if constexpr (MODE != MODE_DENSE) load_rows(ti_iss, total_q > 0, rows_cur);
    // issue the global loads of the next slab of the sequence into set j -- OOB (zeros) past its end -- after
    // the gather rows of the slab that follows it (rows are per tile, re-read per slab: L1 hits, and no load
    // waits on a runtime condition)
    auto issue = [&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const bool valid = iss_i < my_tiles;
      const bool last = iss_kt + 1 == nk;
      int rows_nxt[A_IT];
      if constexpr (MODE != MODE_DENSE) load_rows(last ? ti_fol : ti_iss, last ? iss_i + 1 < my_tiles : valid, rows_nxt);
      if (iss_kt == 0) {  // a new tile: row offsets of its staged rows
#pragma unroll
        for (int r = 0; r < A_IT; ++r) {
          const int m = ti_iss.m0 + prow + 32 * r;
          bool ok = valid && m < ti_iss.M;
          int row = m;
          if constexpr (MODE != MODE_DENSE) {
            row = rows_cur[r];
            ok = ok && row >= 0;
          }
          abase[r] = ok ? (unsigned)row * lda32 * 4u : OOB;
        }
#pragma unroll
        for (int r = 0; r < W_IT; ++r) {
          const int n = ti_iss.n0 + prow + 32 * r;
          wbase[r] = (valid && n < p.N) ? (unsigned)n * ldw32 * 4u : OOB;
        }
      }
      const int k = iss_kt * BK + pcol;
      const unsigned k4 = k < K ? (unsigned)k * 4u : OOB;  // (OOB + a row offset stays past the extent)
#pragma unroll
      for (int r = 0; r < A_IT; ++r) ra[j][r] = bload4(rA, SFX_WS_ABLATE == 2 ? OOB : abase[r] + k4);
      const __amdgpu_buffer_rsrc_t rW = rsrc(ti_iss.Wsp);
#pragma unroll
      for (int r = 0; r < W_IT; ++r)
        rw[j][r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rW, SFX_WS_ABLATE == 2 ? OOB : wbase[r] + k4, 0, 0));
      if constexpr (MODE != MODE_DENSE) {
#pragma unroll
        for (int r = 0; r < A_IT; ++r) rows_cur[r] = rows_nxt[r];
      }
      if (last) {
        iss_kt = 0;
        ++iss_i;
        ti_iss = ti_fol;
        ti_fol = tile_geo<BM, BN, MODE>(p, g, lid + (iss_i + 1) * nwg, tiles_n);
      } else {
        ++iss_kt;
      }
    };

    // store side: slab st_q = (st_i, st_kt) into stage st_s; per-row scale state of tile st_i
    int st_q = 0, st_i = 0, st_kt = 0, st_s = 0;
    int erow[A_IT];
    float srow[A_IT], thr[A_IT];
#pragma unroll
    for (int r = 0; r < A_IT; ++r) { erow[r] = E_UNSET; srow[r] = 1.f; thr[r] = 0.f; }
    auto store = [&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      char* base = smem + st_s * L::STAGE;
      float m[A_IT];
      bool over = false;
#pragma unroll
      for (int r = 0; r < A_IT; ++r) {
        const float4 v = ra[j][r];
        m[r] = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
        over |= m[r] > thr[r];
      }
      if (st_kt == 0 || __builtin_amdgcn_ballot_w64(over) != 0) {
        // slow path (a tile's first slab, a row's first non-zero slab, or a slab that would overflow fp16):
        // row maxima over the 8 lanes of each row, new exponents, rescale factors and 1/s
        bool dec = false;
        float* inv = s_inv + (st_i & 1) * BM;
#pragma unroll
        for (int r = 0; r < A_IT; ++r) {
          const float mr = max8(m[r]);
          int e = st_kt == 0 ? E_UNSET : erow[r];
          float fac = 1.f;
          bool chg = st_kt == 0;
          if (mr > 0.f && mr <= 3.4028235e38f) {
            if (e == E_UNSET) {  // the row's accumulators are still zero: no rescale
              e = row_exp(mr);
              chg = true;
            } else if (mr * srow[r] > 65504.f) {
              const int e2 = row_exp(mr);
              fac = ldexpf(1.f, e2 - e);
              e = e2;
              chg = true;
              dec = true;
            }
          }
          erow[r] = e;
          const bool set = e != E_UNSET;
          srow[r] = set ? ldexpf(1.f, e) : 1.f;
          thr[r] = set ? ldexpf(65504.f, -e) : 0.f;
          if (pc4 == 0) {
            s_fac[st_s * BM + prow + 32 * r] = fac;
            if (chg) inv[prow + 32 * r] = set ? ldexpf(1.f, -e) : 1.f;
          }
        }
        if (__builtin_amdgcn_ballot_w64(dec) != 0 && lane == 0) s_flag[st_s * 4 + pw] = st_q + 1;
      }
#pragma unroll
      for (int r = 0; r < A_IT; ++r) {
        uint2 t[2];
        split2h(ra[j][r], srow[r], t);
        *reinterpret_cast<uint2*>(base + lds_off + 2048 * r) = t[0];
        *reinterpret_cast<uint2*>(base + L::TA + lds_off + 2048 * r) = t[1];
      }
#pragma unroll
      for (int r = 0; r < W_IT; ++r) {
        *reinterpret_cast<uint2*>(base + 2 * L::TA + lds_off + 2048 * r) = make_uint2(rw[j][r].x, rw[j][r].y);
        *reinterpret_cast<uint2*>(base + 2 * L::TA + L::TW + lds_off + 2048 * r) = make_uint2(rw[j][r].z, rw[j][r].w);
      }
      ++st_q;
      st_s = st_s + 1 == NS ? 0 : st_s + 1;
      if (++st_kt == nk) {
        st_kt = 0;
        ++st_i;
      }
    };

    // ---- epilogue of the previous tile, from the staging area (the consumers stage a finished tile's
    // pre-activation values v = acc * 1/s_row * 1/s_W * scale + bias * scale + shift in the round of its last
    // slab).  The producers spread it over the next tile's first nk - 1 rounds (the staging area is rewritten
    // in the nk-th), EPI_ITEMS float4 items per thread, row-major and coalesced: pre-activation copy,
    // activation, row scale, activation derivative, copy, residual, store.
    const unsigned ldy32 = (unsigned)p.ldy, ldr32 = (unsigned)p.ldr, ldp32 = (unsigned)p.ldypre;
    const int per_round = (EPI_ITEMS + nk - 2) / (nk - 1);
    int epi_i = -1, epi_done = EPI_ITEMS;  // tile (local index) whose epilogue is pending, items done
    TileGeo ti_epi{};
    auto epi_items = [&](int count) __attribute__((always_inline)) {
      float* Y = p.Y + g * p.gY;
      const __amdgpu_buffer_rsrc_t rY = rsrc(Y);
#pragma unroll 1
      for (int c = 0; c < count && epi_done < EPI_ITEMS; ++c, ++epi_done) {
        const int it = epi_done * 256 + pt;
        const int row = it / (BN / 4), c4 = it - row * (BN / 4);
        const float4 sv = *reinterpret_cast<const float4*>(s_stg + row * L::SLD + c4 * 4);
        float v[4] = {sv.x, sv.y, sv.z, sv.w};
        const int mt = ti_epi.m0 + row;
        if (mt >= ti_epi.M) continue;
        const int m = ti_epi.out_rows ? ti_epi.out_rows[mt] : mt;
        const int n0 = ti_epi.n0 + c4 * 4;
        if (n0 >= p.N) continue;
        // 16-byte accesses where every operand allows them (p.epi_vec: N and leading dimensions multiples of 4,
        // 16-byte aligned bases), else per element
        auto ld4 = [&](const float* base, unsigned ld, int r) -> float4 {
          const __amdgpu_buffer_rsrc_t rb = rsrc(base);
          if (p.epi_vec) return bload4(rb, ((unsigned)r * ld + (unsigned)n0) * 4u);
          float4 t;
          t.x = bload1(rb, ((unsigned)r * ld + (unsigned)n0) * 4u);
          t.y = bload1(rb, n0 + 1 < p.N ? ((unsigned)r * ld + (unsigned)(n0 + 1)) * 4u : OOB);
          t.z = bload1(rb, n0 + 2 < p.N ? ((unsigned)r * ld + (unsigned)(n0 + 2)) * 4u : OOB);
          t.w = bload1(rb, n0 + 3 < p.N ? ((unsigned)r * ld + (unsigned)(n0 + 3)) * 4u : OOB);
          return t;
        };
        auto st4 = [&](__amdgpu_buffer_rsrc_t rb, unsigned ld, const float (&x)[4]) {
          if (p.epi_vec) {
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const floatx4 t = {x[0], x[1], x[2], x[3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, t), rb, ((unsigned)m * ld + (unsigned)n0) * 4u,
                                                   0, 0);
            return;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e)
            bstore1(rb, n0 + e < p.N ? ((unsigned)m * ld + (unsigned)(n0 + e)) * 4u : OOB, x[e]);
        };
        float4 rv;
        if (p.R) rv = ld4(p.R, ldr32, p.ridx ? p.ridx[m] : m);
        if (p.Ypre && p.pre_before_act) st4(rsrc(p.Ypre), ldp32, v);
        if (p.act != ACT_NONE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool do_act = n0 + e < p.act_ncols;
            if (p.act == ACT_GELU) v[e] = do_act ? gelu_erf(v[e]) : v[e];
            else if (p.act == ACT_RELU) v[e] = do_act ? fmaxf(v[e], 0.f) : v[e];
            else v[e] = do_act ? tanhf(v[e]) : v[e];
          }
        }
        if (p.rowscale) {
          const float rs = p.rowscale[m];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= rs;
        }
        if (p.dact) {
          const float4 pr = ld4(p.dact_pre, (unsigned)p.ld_dact, m);
          const float pre[4] = {pr.x, pr.y, pr.z, pr.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = n0 + e < p.act_ncols ? v[e] * dact_grad(p.dact, pre[e]) : v[e];
        }
        if (p.Ypre && !p.pre_before_act) st4(rsrc(p.Ypre), ldp32, v);
        if (p.R) {
          v[0] += rv.x;
          v[1] += rv.y;
          v[2] += rv.z;
          v[3] += rv.w;
        }
        if (p.y_amax) {
#pragma unroll
          for (int e = 0; e < 4; ++e) ymax = fmaxf(ymax, n0 + e < p.N ? fabsf(v[e]) : 0.f);
        }
        st4(rY, ldy32, v);
      }
    };
    // round q (0-based, after the prologue barrier): a tile staged in round q - 1 becomes pending; rounds
    // q .. q + nk - 2 run its items
    auto epi_round = [&](int q) __attribute__((always_inline)) {
      if constexpr (MODE == MODE_PAIR) return;
      if (q > 0 && q <= total_q && q % nk == 0) {
        epi_i = q / nk - 1;
        epi_done = 0;
        ti_epi = tile_geo<BM, BN, MODE>(p, g, lid + epi_i * nwg, tiles_n);
      }
      if (epi_done < EPI_ITEMS) epi_items(per_round);
    };

    // NSET register sets: slab s is issued NSET - 1 barrier rounds before it is split and stored.  The slab
    // sequence is padded to a multiple of NSET: the loop body handles NSET slabs with compile-time set indices
    // and no exit in between (so hipcc's wait counts stay exact); a padding slab issues only OOB loads and
    // stores into a stage that nobody reads afterwards.
    static_for<0, NSET>([&](auto jc) { issue(jc); });
    store(std::integral_constant<int, 0>{});
    __syncthreads();
#if SFX_WS_TRACE
    unsigned long long pt_iss = 0, pt_st = 0, pt_epi = 0, pt_bar = 0;
#endif
    for (int q = 0; q < total_qp; q += NSET) {
      static_for<0, NSET>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        WS_T(t0);
        issue(jc);                                             // set j: slab q + j + NSET
        WS_T(t1);
        store(std::integral_constant<int, (j + 1) % NSET>{});  // slab q + j + 1
        WS_T(t2);
        epi_round(q + j);
        WS_T(t3);
        __syncthreads();
#if SFX_WS_TRACE
        WS_T(t4);
        pt_iss += t1 - t0; pt_st += t2 - t1; pt_epi += t3 - t2; pt_bar += t4 - t3;
#endif
      });
    }
#if SFX_WS_TRACE
    if (tid == WS_CONS * 64) {
      atomicAdd(&g_ws_trace[0], pt_iss); atomicAdd(&g_ws_trace[1], pt_st);
      atomicAdd(&g_ws_trace[2], pt_epi); atomicAdd(&g_ws_trace[3], pt_bar);
      atomicAdd(&g_ws_trace[8], (unsigned long long)total_qp);
    }
#endif
    // the last tile's epilogue (staged in round total_q - 1)
    if (MODE != MODE_PAIR && total_q > 0) {
      if (total_qp == total_q) {  // its items were not started in a padding round
        epi_i = my_tiles - 1;
        epi_done = 0;
        ti_epi = tile_geo<BM, BN, MODE>(p, g, lid + epi_i * nwg, tiles_n);
      }
      epi_items(EPI_ITEMS);
    }
  } else {
    // ------------------------------------------------------------------ consumers
    const int wm = wid / WGN, wn = wid % WGN;
    const int h = lane >> 5, l32 = lane & 31;
    const float* bias = p.bias ? p.bias + g * p.gB : nullptr;
    floatx16 acc[MB][NB];
    TileGeo ti{};
    typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;

    auto compute = [&](int st) __attribute__((always_inline)) {
      const char* base = smem + st * L::STAGE;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        f16x8 af[MB][2], wf[NB][2];
#pragma unroll
        for (int qd = 0; qd < 2; ++qd) {
#pragma unroll
          for (int a = 0; a < MB; ++a)
            af[a][qd] = __builtin_bit_cast(
                f16x8, *reinterpret_cast<const uint4*>(base + qd * L::TA + swz(wm * WM + a * 32 + l32, 4 * s + 2 * h)));
#pragma unroll
          for (int b = 0; b < NB; ++b)
            wf[b][qd] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(
                                                      base + 2 * L::TA + qd * L::TW + swz(wn * WN + b * 32 + l32, 4 * s + 2 * h)));
        }
        // smallest terms first; consecutive MFMAs write different accumulators
        constexpr int QA[3] = {1, 0, 0}, QW[3] = {0, 1, 0};
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int a = 0; a < MB; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[a][QA[j]], wf[b][QW[j]], acc[a][b], 0, 0, 0);
      }
    };
    // accumulator rows of 8-row group gq (staged by producer wave gq) times v[row]
    auto scale_group = [&](const float* v, int gq) __attribute__((always_inline)) {
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        const float4 f = *reinterpret_cast<const float4*>(v + wm * WM + a * 32 + 8 * gq + 4 * h);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          acc[a][b][4 * gq + 0] *= f.x;
          acc[a][b][4 * gq + 1] *= f.y;
          acc[a][b][4 * gq + 2] *= f.z;
          acc[a][b][4 * gq + 3] *= f.w;
        }
      }
    };
    // stage the finished tile: v = acc * 1/s_row * (1/s_W scale)[col] + (bias scale + shift)[col]
    auto stage_tile = [&](const float* inv) __attribute__((always_inline)) {
      const __amdgpu_buffer_rsrc_t rB = rsrc(bias ? bias : p.A);
      const __amdgpu_buffer_rsrc_t rSc = rsrc(p.scale ? p.scale : p.A);
      const __amdgpu_buffer_rsrc_t rH = rsrc(p.shift ? p.shift : p.A);
      const __amdgpu_buffer_rsrc_t rV = rsrc(ti.winv ? ti.winv : p.A);
      float c1[NB], c0[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int n = ti.n0 + wn * WN + b * 32 + l32;
        const unsigned off = n < p.N ? (unsigned)n * 4u : OOB;
        const float bv = bload1(rB, bias ? off : OOB);
        const float sv = p.scale ? bload1(rSc, off) : 1.f;
        const float hv = bload1(rH, p.shift ? off : OOB);
        const float wv = ti.winv ? bload1(rV, off) : 1.f;
        c1[b] = sv * wv;
        c0[b] = MODE == MODE_PAIR ? 0.f : bv * sv + hv;
      }
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int row = wm * WM + a * 32 + 8 * gq + 4 * h;
          const float4 f = *reinterpret_cast<const float4*>(inv + row);
          const float fr[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const int col = wn * WN + b * 32 + l32;
#pragma unroll
            for (int i = 0; i < 4; ++i)
              s_stg[(row + i) * L::SLD + col] = __builtin_fmaf(acc[a][b][4 * gq + i] * fr[i], c1[b], c0[b]);
          }
        }
    };

    // pair mode (one neighbour offset's partial sums): unscale and add atomically into the output rows straight
    // from the accumulators (32 lanes = 128 contiguous bytes per atomic instruction row)
    auto pair_epilogue = [&](const float* inv) __attribute__((always_inline)) {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) scale_group(inv, gq);
      const __amdgpu_buffer_rsrc_t rY = rsrc(p.Y);
      const __amdgpu_buffer_rsrc_t rO = rsrc(ti.out_rows);
      const __amdgpu_buffer_rsrc_t rV = rsrc(ti.winv ? ti.winv : p.A);
      const unsigned ldy32 = (unsigned)p.ldy;
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        int o[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mt = ti.m0 + wm * WM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          o[r] = mt < ti.M ? bload1i(rO, (unsigned)mt * 4u) : -1;
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const int n = ti.n0 + wn * WN + b * 32 + l32;
          const bool nok = n < p.N;
          const float c1 = ti.winv ? bload1(rV, nok ? (unsigned)n * 4u : OOB) : 1.f;
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(
                acc[a][b][r] * c1, rY, (nok && o[r] >= 0) ? ((unsigned)o[r] * ldy32 + (unsigned)n) * 4u : OOB, 0, 0);
        }
      }
    };

    __syncthreads();
    int c_i = 0, c_kt = 0, st = 0;
#if SFX_WS_TRACE
    unsigned long long ct_pre = 0, ct_mma = 0, ct_stg = 0, ct_bar = 0;
#endif
    for (int q = 0; q < total_qp; ++q) {
      WS_T(c0);
#if SFX_WS_TRACE
      unsigned long long c1 = c0, c2 = c0, c3 = c0;
#endif
      if (q < total_q) {
        if (c_kt == 0) {
          ti = tile_geo<BM, BN, MODE>(p, g, lid + c_i * nwg, tiles_n);
#pragma unroll
          for (int a = 0; a < MB; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
              for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
        } else {
          const int4 fl = *reinterpret_cast<const int4*>(s_flag + st * 4);
          const int stamp = q + 1;
          if (__builtin_amdgcn_readfirstlane(fl.x) == stamp) scale_group(s_fac + st * BM, 0);
          if (__builtin_amdgcn_readfirstlane(fl.y) == stamp) scale_group(s_fac + st * BM, 1);
          if (__builtin_amdgcn_readfirstlane(fl.z) == stamp) scale_group(s_fac + st * BM, 2);
          if (__builtin_amdgcn_readfirstlane(fl.w) == stamp) scale_group(s_fac + st * BM, 3);
        }
#if SFX_WS_TRACE
        c1 = __builtin_readcyclecounter();
#endif
        if (SFX_WS_ABLATE != 1) compute(st);
#if SFX_WS_TRACE
        c2 = __builtin_readcyclecounter();
#endif
        if (c_kt == nk - 1) {
          if constexpr (MODE == MODE_PAIR) pair_epilogue(s_inv + (c_i & 1) * BM);
          else stage_tile(s_inv + (c_i & 1) * BM);
        }
#if SFX_WS_TRACE
        c3 = __builtin_readcyclecounter();
#endif
        st = st + 1 == NS ? 0 : st + 1;
        if (++c_kt == nk) {
          c_kt = 0;
          ++c_i;
        }
      }
      __syncthreads();
#if SFX_WS_TRACE
      WS_T(c4);
      ct_pre += c1 - c0; ct_mma += c2 - c1; ct_stg += c3 - c2; ct_bar += c4 - c3;
#endif
    }
#if SFX_WS_TRACE
    if (tid == 0) {
      atomicAdd(&g_ws_trace[4], ct_pre); atomicAdd(&g_ws_trace[5], ct_mma);
      atomicAdd(&g_ws_trace[6], ct_stg); atomicAdd(&g_ws_trace[7], ct_bar);
    }
#endif
  }
  if (p.y_amax) sfx::publish_amax(ymax, p.y_amax, p.y_tag, reinterpret_cast<float*>(smem + WsLds<BM, BN, NS>::YW));
}

// ---- weight pre-split: one wave per row -------------------------------------------------------------------
// dst row n (contiguous, cols elements): per 4-element group, fp16 h terms then fp16 l terms of W[n, k] * 2^e_n,
// with e_n putting the row's maximum in [2^14, 2^15) (0 for an all-zero row); inv[n] = 2^-e_n.
__global__ void __launch_bounds__(256) weight_split_kernel(int rows, int cols, const float* __restrict__ src,
                                                           long long ld, float* __restrict__ dst,
                                                           float* __restrict__ inv) {
  const int row = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = src + (long long)row * ld;
  float m = 0.f;
  for (int c = lane * 4; c < cols; c += 256) {
    const float4 v = *reinterpret_cast<const float4*>(s + c);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  m = sfx::wave_max(m);
  int e = 0;
  if (m > 0.f && m <= 3.4028235e38f) e = row_exp(m) + 2;
  const float sc = ldexpf(1.f, e);
  uint2* d = reinterpret_cast<uint2*>(dst + (long long)row * cols);
  for (int c = lane * 4; c < cols; c += 256) {
    uint2 t[2];
    split2h(*reinterpret_cast<const float4*>(s + c), sc, t);
    d[c / 2] = t[0];
    d[c / 2 + 1] = t[1];
  }
  if (lane == 0) inv[row] = ldexpf(1.f, -e);
}

int ws_num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

// M-tiles of a launch (pair mode: per-slice rounding, fills slice_tile_off)
int ws_tiles_m(GemmArgs& a, int BM) {
  if (!a.pair_mode) return (int)sfx::ceil_div(a.M, BM);
  int t = 0;
  for (int k = 0; k < a.num_slices; ++k) {
    a.slice_tile_off[k] = t;
    t += (a.slice_pair_off[k + 1] - a.slice_pair_off[k] + BM - 1) / BM;
  }
  a.slice_tile_off[a.num_slices] = t;
  return t;
}

constexpr int WS_NS = 2;

template <int BM, int BN, int WGM, int MODE>
void ws_launch(GemmArgs a, int groups, hipStream_t st) {
  const int tiles_m = ws_tiles_m(a, BM);
  const int tiles_n = (int)sfx::ceil_div(a.N, BN);
  const int total = tiles_m * tiles_n;
  const int slots = ws_num_cus() / groups > 0 ? ws_num_cus() / groups : 1;
  const int per = (total + slots - 1) / slots;  // balanced: every workgroup gets per or per - 1 tiles
  const int grid_x = total > 0 ? (total + per - 1) / per : 1;
  // register sets of the producers' prefetch: as many as ~160 VGPRs hold (16 B per staged group and set)
  constexpr int NSET = (BM + BN) / 32 * 4 <= 32 ? 4 : 3;
  gemm_ws_kernel<BM, BN, WGM, MODE, WS_NS, NSET><<<dim3(grid_x, 1, groups), WS_THREADS, 0, st>>>(a, tiles_n, total);
}

struct WsCfg {
  int bm, bn;
};
// (64 accumulators per consumer lane: the 128-accumulator shapes spill in the epilogue)
constexpr WsCfg kWs[] = {{128, 128}, {256, 64}};
constexpr int kNumWs = sizeof(kWs) / sizeof(kWs[0]);

int ws_forced() {
  static int f = -2;
  if (f == -2) {
    const char* e = getenv("SFX_GEMM_WS_CFG");
    f = (e && *e) ? atoi(e) : -1;
    if (f >= kNumWs) f = -1;
  }
  return f;
}

// rounds of per-CU tiles x (slabs + ~1 slab of epilogue) x tile area (the MFMA work of a round is the tile's)
int ws_pick(GemmArgs& a, int groups) {
  if (ws_forced() >= 0) return ws_forced();
  const long long nk = sfx::ceil_div(a.K, BK);
  const long long slots = ws_num_cus() / groups > 0 ? ws_num_cus() / groups : 1;
  int best = 0;
  double best_cost = 1e300;
  for (int c = 0; c < kNumWs; ++c) {
    const long long tiles = (long long)ws_tiles_m(a, kWs[c].bm) * sfx::ceil_div(a.N, kWs[c].bn) * groups;
    const long long rounds = (tiles + slots - 1) / slots;
    // smaller tiles pay more LDS traffic and epilogue per MFMA: weight by a mild efficiency factor
    const double eff = (kWs[c].bm * kWs[c].bn >= 256 * 128) ? 1.0 : (kWs[c].bm * kWs[c].bn >= 128 * 128 ? 0.9 : 0.85);
    const double cost = (double)rounds * (nk + 1.5) * kWs[c].bm * kWs[c].bn / eff;
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  ws_tiles_m(a, kWs[best].bm);
  return best;
}

template <int MODE>
void ws_dispatch(GemmArgs a, int groups, hipStream_t st) {
  switch (ws_pick(a, groups)) {
    case 0: ws_launch<128, 128, 2, MODE>(a, groups, st); break;
    default: ws_launch<256, 64, 4, MODE>(a, groups, st); break;
  }
}

}  // namespace

namespace sfxg {

bool ws_enabled() {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("SFX_GEMM_WS");  // opt-in (measured slower than the general kernel on config B)
    en = (e && *e == '1') ? 1 : 0;
  }
  return en == 1;
}

bool launch_ws(const GemmArgs& a0, int groups, hipStream_t st) {
  if (!ws_enabled() || a0.split != 2 || a0.sk || !a0.Wsp || (a0.gidx && !a0.pair_mode && a0.S != 1)) return false;
  GemmArgs a = a0;
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  a.epi_vec = a.N % 4 == 0 && a.ldy % 4 == 0 && al(a.Y) && a.gY % 4 == 0 &&
              (!a.R || (a.ldr % 4 == 0 && al(a.R))) && (!a.Ypre || (a.ldypre % 4 == 0 && al(a.Ypre))) &&
              (!a.dact || (a.ld_dact % 4 == 0 && al(a.dact_pre)));
  if (a.pair_mode)
    ws_dispatch<MODE_PAIR>(a, groups, st);
  else if (!a.gidx)
    ws_dispatch<MODE_DENSE>(a, groups, st);
  else
    ws_dispatch<MODE_GATHER1>(a, groups, st);
  return true;
}

}  // namespace sfxg

extern "C" int sfx_weight_split(int rows, int cols, const float* w, long long ld, float* w_split, float* w_inv,
                                void* stream) {
  SFX_REQUIRE(rows >= 0 && cols > 0 && cols % 4 == 0 && ld >= cols && ld % 4 == 0,
              "sfx_weight_split: bad sizes (cols and ld must be multiples of 4)");
  if (rows == 0) return SFX_OK;
  SFX_REQUIRE(w && w_split && w_inv, "sfx_weight_split: null buffer");
  SFX_REQUIRE((reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(w_split) & 15) == 0,
              "sfx_weight_split: buffers must be 16-byte aligned");
  weight_split_kernel<<<sfx::ceil_div(rows, 4), 256, 0, sfx::as_stream(stream)>>>(rows, cols, w, ld, w_split, w_inv);
  return sfx::check_launch("sfx_weight_split");
}

#if SFX_WS_TRACE
extern "C" int sfx_ws_trace(unsigned long long* out, int reset) {
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ws_trace), sizeof(unsigned long long) * 16);
  if (reset) {
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_ws_trace), z, sizeof(z));
  }
  return 0;
}
#endif
