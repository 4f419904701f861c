// fp32-accurate GEMM on pre-split operands with an LDS-DMA pipeline (the "deep" GEMM of the large refiner
// shapes: K >= 128, N >= 128 -- stage 3 / 4 linears and SubM convs, 37759 x 256..1024 x 256..1024 on config B).
//
//   Y[m, n] = act((sum_k A'[m, k] W[n, k]) * sa[m] * sw[n] + bias[n]) (* scale[n] + shift[n]) + R[.., n]
//
// Operands arrive pre-split (sfx_split_rows): every row r of a fp32 matrix X becomes two fp16 planes
// H[r][k] = fp16(X[r][k] * 2^e_r), L[r][k] = fp16(X[r][k] * 2^e_r - H[r][k]) and inv[r] = 2^-e_r, with e_r putting
// the row maximum in [2^14, 2^15) -- the same fp16x2 terms as the in-kernel split of gemm.hip (h*h + h*l + l*h per
// 32x32x16 block on v_mfma_f32_32x32x16_f16, fp32 accumulation: the error of fp32 arithmetic).  Rows are padded to
// Kp (a multiple of 32, zero tail) so every 64-byte k-segment is whole.
//
// Why a second kernel: gemm.hip stages both operands through registers one 32-deep slab ahead (split on the
// store), so each slab's global-load latency is covered by only one slab of MFMAs; SQ counters put its waves
// 38-53 % in s_waitcnt / barrier waits (profiles/r03_mlp_sq_counters.txt).  Here nothing is split in the loop:
// both operands go global -> LDS by buffer_load ... lds (per-lane source rows, so gathered A rows -- SubM pair
// lists, centre neighbours -- need no register pass), three stages in flight in an LDS ring, one raw barrier per
// stage, counted vmcnt.  Tile 256 x 128 (8 waves, 64 x 64 each: 12 MFMAs per 16-deep k-step), 48 KB per stage,
// 144 KB ring: 256 x 128 x 32 MACs x 3 terms per 48 KB = 31 B/clk per CU at the full MFMA rate.
#include <cstdlib>
#include <type_traits>

#include "gemm_common.h"

// ablation builds only (tools/build_variant.sh): 1 no MFMA, 2 no operand DMA, 4 stores dropped, 8 no fragment reads,
// 16 empty kernel, 32 no epilogue, 64 no store instructions (stamps: vmcnt counts then over-wait), 128 no
// staggered units
#ifndef G2_ABL
#define G2_ABL 0
#endif
// diagnostic build (-DG2_STAMP=1): per wave s_memtime totals (loop, waits, epilogues) into the buffer set by
// sfx_gemm2_stamps
#ifndef G2_STAMP
#define G2_STAMP 0
#endif
#if G2_STAMP
__device__ unsigned long long* g2_stamp_buf;
#define STAMP() __builtin_amdgcn_s_memtime()
#endif

namespace {

using namespace sfxg;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int G2_BM = 256, G2_BN = 128, G2_BK = 32, G2_NW = 8, G2_STAGES = 3;
constexpr int G2_A_BYTES = 2 * G2_BM * 64, G2_W_BYTES = 2 * G2_BN * 64;
constexpr int G2_STAGE_BYTES = G2_A_BYTES + G2_W_BYTES;          // 48 KB
constexpr int G2_RING_BYTES = G2_STAGES * G2_STAGE_BYTES;         // 144 KB
constexpr int G2_A_PIECES = G2_A_BYTES / 1024 / G2_NW;             // 1-KB DMA pieces per wave per stage: 4
constexpr int G2_W_PIECES = G2_W_BYTES / 1024 / G2_NW;             // 2
constexpr int G2_PIECES = G2_A_PIECES + G2_W_PIECES;
// per-tile constants, three buffers (tile % 3): column constants winv / bias / scale / shift [4][128] floats,
// A-row 1/s [256] floats, A-row indices [256] ints (gather / pair modes)
constexpr int G2_TC_BYTES = 4096, G2_TC_COLS = 0, G2_TC_AINV = 2048, G2_TC_IDX = 3072;
constexpr int G2_LDS_BYTES = G2_RING_BYTES + 3 * G2_TC_BYTES;      // 156 KB
constexpr int G2_EPI_STORES = 16;  // buffer_store_dwordx4 per lane per tile epilogue (counted by the stage waits)

enum G2Mode { G2_DENSE = 0, G2_GATHER = 1, G2_PAIR = 2 };
// epilogue kinds (template): bias / BN affine; + erf GELU on columns < act_ncols; bias + residual rows
enum G2Epi { G2_EPI_AFFINE = 0, G2_EPI_GELU = 1, G2_EPI_RES = 2 };

struct G2Args {
  int M, N, Kp;                 // Kp: padded K (multiple of 32, >= 64)
  const _Float16* A;            // pre-split A planes: A[q * a_plane + row * Kp + k]
  long long a_plane;
  const float* ainv;            // [a_rows] 1/s
  int a_rows;
  const int* gidx;              // gather: A row of output row m = gidx[m * gstride] (or -1); pair: pair_in
  int gstride;
  const _Float16* W;            // pre-split W planes [N][Kp] (pair mode: [27][N][Kp])
  long long w_plane;
  const float* winv;            // [N] (pair mode: [27][N])
  const float* bias;            // the column arrays must be 16-byte aligned; absent ones point at winv
  const float* scale;
  const float* shift;
  int has_bias, has_scale, has_shift;
  int act, act_ncols;
  const float* R;               // residual (16-byte aligned rows)
  long long ldr;
  float* Y;
  long long ldy;
  unsigned long long* y_amax;
  unsigned y_tag;
  int num_slices;               // pair mode: 27 slices of the flat tile list, outputs stored at row `pair index`
  int slice_tile_off[28];
  int slice_pair_off[28];
};

struct G2Tile {
  int m0, Mt, n0, pbase, sl;
};

template <int MODE>
__device__ __forceinline__ G2Tile g2_tile(const G2Args& p, int t, int tiles_n) {
  G2Tile ti;
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  ti.n0 = tn * G2_BN;
  ti.m0 = tm * G2_BM;
  ti.Mt = p.M;
  ti.pbase = 0;
  ti.sl = 0;
  if constexpr (MODE == G2_PAIR) {
    int sl = 0;
    for (int q = 1; q < p.num_slices; ++q)
      if (p.slice_tile_off[q] <= tm) sl = q;
    ti.sl = sl;
    ti.pbase = p.slice_pair_off[sl];
    ti.Mt = p.slice_pair_off[sl + 1] - ti.pbase;
    ti.m0 = (tm - p.slice_tile_off[sl]) * G2_BM;
  }
  return ti;
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// LDS-DMA as inline asm: the compiler neither counts these loads nor sees their LDS writes, so it inserts no
// hazard waits of its own around them (its builtin form costs a vmcnt(0) whenever a register that served as a DMA
// address is reused); the stage waits below count them explicitly.  M0 is saved and restored around each.
struct Srd {
  u32x4 v;
};
__device__ __forceinline__ Srd make_srd(const void* base, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  Srd r;
  r.v[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
  r.v[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) & 0xffffu;
  r.v[2] = __builtin_amdgcn_readfirstlane(bytes);
  r.v[3] = (unsigned)RSRC_FLAGS;
  return r;
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long long)((__attribute__((address_space(3))) const char*)p));
}
__device__ __forceinline__ void dma_b128(const Srd& srd, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(srd.v), "s"(lds)
               : "memory");
}
__device__ __forceinline__ void dma_b32(const Srd& srd, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(srd.v), "s"(lds)
               : "memory");
}
__device__ __forceinline__ void dma_g128(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

// Persistent: one workgroup per CU walks its tiles (XCD-contiguous ranges, N-tiles of one row block back to back)
// as ONE stream of 32-deep stages: stage g + 2 is issued while stage g is computed, across tile boundaries, so
// a tile's first loads overlap the previous tile's last MFMAs and epilogue.  MFMA operands are swapped (W rows
// as the A operand), so each lane's accumulators hold 4 consecutive output columns: 16-byte stores.
template <int MODE, int EPI>
__global__ void __launch_bounds__(512, 1) gemm2_kernel(G2Args p, int tiles_n, int total) {
  __shared__ __attribute__((aligned(16))) char lds[G2_LDS_BYTES];
  if (G2_ABL & 16) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;  // 4 x 2 waves, 64 x 64 each
  const int h = lane >> 5, r32 = lane & 31;

  // ---- this workgroup's tiles ----
  const int P = (int)gridDim.x;
  int tstart, tstep, tend;
  if (P >= total) {  // one tile per workgroup: XCD-contiguous numbering
    const int q = P / 8, r = P % 8, x = (int)blockIdx.x % 8;
    tstart = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (int)blockIdx.x / 8;
    tstep = 1;
    tend = tstart + 1;
  } else {  // P is a multiple of 8: XCD x owns tiles [total x / 8, total (x + 1) / 8)
    const int x = (int)blockIdx.x % 8, j = (int)blockIdx.x / 8, px = P / 8;
    const int lo = (int)((long long)total * x / 8), hi = (int)((long long)total * (x + 1) / 8);
    tstart = lo + j;
    tstep = px;
    tend = hi;
  }
  if (tstart >= min(tend, total)) return;
  tend = min(tend, total);
  const int n_my = (tend - tstart + tstep - 1) / tstep;
  const int nk = p.Kp / G2_BK;
  const int S = n_my * nk;

  const Srd rA = make_srd(p.A, OOB), rW = make_srd(p.W, OOB), rI = make_srd(p.gidx, OOB);
  const Srd rAi = make_srd(p.ainv, (unsigned)p.a_rows * 4u);
  const unsigned a_plane_b = (unsigned)(p.a_plane * 2), w_plane_b = (unsigned)(p.w_plane * 2);
  const unsigned kp_b = (unsigned)p.Kp * 2u;
  char* const tcb = lds + G2_RING_BYTES;

  // idx of tile `loc` (gather / pair): 4 dword DMAs of 64 rows, issued by waves 6, 7, 0, 1
  auto issue_idx = [&](int loc) {
    if constexpr (MODE != G2_DENSE) {
      const int jw = (wid + 2) & 7;  // waves 6, 7, 0, 1 -> pieces 0..3
      if (jw < 4) {
        const G2Tile ti = g2_tile<MODE>(p, tstart + loc * tstep, tiles_n);
        const int m = ti.m0 + jw * 64 + lane;
        const unsigned off = m < ti.Mt ? (unsigned)(ti.pbase + m) * (unsigned)p.gstride * 4u : OOB;
        dma_b32(rI, off, lds_addr(tcb + (loc % 3) * G2_TC_BYTES + G2_TC_IDX + jw * 256));
      }
    }
  };

  // ---- issue side: stage stream state ----
  int i_loc = 0, i_kt = 0;
  G2Tile it{};
  unsigned a_src[G2_A_PIECES], w_src[G2_W_PIECES];
  unsigned cur_off[G2_PIECES];  // this issue's per-lane source offsets (A pieces, then W pieces)
  char* cur_st = lds;
  // prep(g): stage g's sources (on a new tile also its row sources, constants and the next tile's indices)
  auto prep = [&](int g) {
    if (i_kt == 0) {  // a new tile: its row sources, its constants, the next tile's indices
      it = g2_tile<MODE>(p, tstart + i_loc * tstep, tiles_n);
      const char* idx = tcb + (i_loc % 3) * G2_TC_BYTES + G2_TC_IDX;
#pragma unroll
      for (int i = 0; i < G2_A_PIECES; ++i) {
        const int piece = wid * G2_A_PIECES + i;  // 0..31: term piece / 16, row block piece % 16
        const int q = piece >> 4, r = (piece & 15) * 16 + (lane >> 2);
        const int c = (lane & 3) ^ ((r >> 2) & 3);
        const int m = it.m0 + r;
        int src = m;
        if constexpr (MODE != G2_DENSE) src = reinterpret_cast<const int*>(idx)[r];
        a_src[i] = (m < it.Mt && src >= 0) ? (unsigned)q * a_plane_b + (unsigned)src * kp_b + (unsigned)c * 16u : OOB;
      }
      const unsigned woff_b = (unsigned)it.sl * (unsigned)p.N * kp_b;
#pragma unroll
      for (int i = 0; i < G2_W_PIECES; ++i) {
        const int piece = wid * G2_W_PIECES + i;  // 0..15: term piece / 8, row block piece % 8
        const int q = piece >> 3, r = (piece & 7) * 16 + (lane >> 2);
        const int c = (lane & 3) ^ ((r >> 2) & 3);
        const int n = it.n0 + r;
        w_src[i] = n < p.N ? (unsigned)q * w_plane_b + woff_b + (unsigned)n * kp_b + (unsigned)c * 16u : OOB;
      }
      char* tc = tcb + (i_loc % 3) * G2_TC_BYTES;
      if (wid < 2) {  // column constants: piece wid covers arrays 2 wid, 2 wid + 1 (32 lanes x 16 B each)
        const int arr = 2 * wid + h;
        const float* base = arr == 0 ? p.winv + it.sl * p.N : arr == 1 ? p.bias : arr == 2 ? p.scale : p.shift;
        const int n = it.n0 + 4 * r32;
        dma_g128(base + (n < p.N ? n : 0), lds_addr(tc + G2_TC_COLS + wid * 1024));
      } else if (wid < 6) {  // A-row 1/s: dense one 1-KB piece, gathered four 64-row dword pieces
        if constexpr (MODE == G2_DENSE) {
          if (wid == 2)
            dma_b128(rAi, (unsigned)(it.m0 + 4 * lane) * 4u, lds_addr(tc + G2_TC_AINV));
        } else {
          const int j = wid - 2;
          const int src = reinterpret_cast<const int*>(idx)[j * 64 + lane];
          const int m = it.m0 + j * 64 + lane;
          dma_b32(rAi, (m < it.Mt && src >= 0) ? (unsigned)src * 4u : OOB, lds_addr(tc + G2_TC_AINV + j * 256));
        }
      }
      if (i_loc + 1 < n_my) issue_idx(i_loc + 1);
    }
    cur_st = lds + (g % G2_STAGES) * G2_STAGE_BYTES;
    const unsigned ko = (unsigned)i_kt * 64u;  // 32 k x 2 B
#pragma unroll
    for (int i = 0; i < G2_A_PIECES; ++i) cur_off[i] = a_src[i] == OOB ? OOB : a_src[i] + ko;
#pragma unroll
    for (int i = 0; i < G2_W_PIECES; ++i) cur_off[G2_A_PIECES + i] = w_src[i] == OOB ? OOB : w_src[i] + ko;
    if (++i_kt == nk) {
      i_kt = 0;
      ++i_loc;
    }
  };
  // DMA piece i of the prepared stage (straight-line: interleaved with the MFMAs)
  auto dma = [&](int i) {
    if (G2_ABL & 2) return;
    if (i < G2_A_PIECES)
      dma_b128(rA, cur_off[i], lds_addr(cur_st + (wid * G2_A_PIECES + i) * 1024));
    else
      dma_b128(rW, cur_off[i], lds_addr(cur_st + G2_A_BYTES + (wid * G2_W_PIECES + i - G2_A_PIECES) * 1024));
  };
  auto issue = [&](int g) {
    prep(g);
#pragma unroll
    for (int i = 0; i < G2_PIECES; ++i) dma(i);
  };

  // prologue: the first tile's indices, then stages 0 and 1
#if G2_STAMP
  unsigned long long t_begin = STAMP(), t_wait = 0, t_epi = 0, t_mfma = 0;
#endif
  issue_idx(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  issue(0);
  issue(1);  // S >= nk >= 4

  const __amdgpu_buffer_rsrc_t rY = rsrc(p.Y);
  const __amdgpu_buffer_rsrc_t rR = rsrc(p.R ? p.R : p.Y);
  float ymax = 0.f;
  floatx16 acc0[2][2], acc1[2][2];
  auto swz = [](int r, int c) { return r * 64 + (((c ^ (r >> 2)) & 3) << 4); };

  // Epilogue of a finished tile in 16 units: unit (part, gq) = 4 consecutive columns of one 32 x 32 accumulator block
  // (part = (a, b)) of each wave, one 16-byte store per lane.  The units of tile t run inside the first E2 stages of
  // tile t + 1 (E2 = 8 when the tile has >= 8 stages: 2 units each; else 4: 4 units each), whose accumulators are
  // the other set, so the stores drain under that tile's MFMAs instead of every CU storing a whole tile at once.
  // A unit's residual row piece is loaded at the end of the stage before it (compiler-counted: at the use it waits
  // for every older load, i.e. also for the stage DMA issued one stage earlier, which had a stage of MFMAs to land).
  const int E2 = nk >= 8 ? 8 : 4;
  constexpr bool RES = EPI == G2_EPI_RES;
  // unit u = (part u >> 2, gq u & 3) belongs to stage kt of the next tile
  auto unit_in = [&](int kt, int u) {
    return E2 == 8 ? ((u & 3) == (kt >> 1) && ((u >> 3) == (kt & 1))) : (u & 3) == kt;
  };
  auto res_load = [&](const G2Tile& ct, int part, int gq) -> u32x4 {
    const int a = part >> 1, b = part & 1;
    const int m = ct.m0 + wm * 64 + a * 32 + r32;
    const int n = ct.n0 + wn * 64 + b * 32 + 8 * gq + 4 * h;
    const unsigned off = (m < ct.Mt && n < p.N) ? ((unsigned)m * (unsigned)p.ldr + (unsigned)n) * 4u : OOB;
    return __builtin_amdgcn_raw_buffer_load_b128(rR, off, 0, 0);
  };
  auto epi_unit = [&](floatx16 (&pacc)[2][2], const G2Tile& ct, int cloc, auto uc, u32x4 rvu) {
    constexpr int u = decltype(uc)::value;  // compile-time: the accumulators stay in registers
    constexpr int part = u >> 2, gq = u & 3, a = part >> 1, b = part & 1;
    // opaque per execution: keeps the 16 units' addresses from being hoisted out of the stage loop (registers)
    int m0 = __builtin_amdgcn_readfirstlane(ct.m0), n0 = __builtin_amdgcn_readfirstlane(ct.n0);
    int tco = __builtin_amdgcn_readfirstlane((cloc % 3) * G2_TC_BYTES);
    asm volatile("" : "+s"(m0), "+s"(n0), "+s"(tco));
    const char* tc = tcb + tco;
    const int ml = wm * 64 + a * 32 + r32;
    const int m = m0 + ml;
    const bool mok = m < ct.Mt;
    const float ai = reinterpret_cast<const float*>(tc + G2_TC_AINV)[ml];
    const unsigned yrow = (unsigned)(MODE == G2_PAIR ? ct.pbase + m : m) * (unsigned)p.ldy;
    const int nl = wn * 64 + b * 32 + 8 * gq + 4 * h;
    const int n = n0 + nl;
    // combined column constants (combine_cols): v = acc * ai * cs + cb
    const floatx4 cs = *reinterpret_cast<const floatx4*>(tc + G2_TC_COLS + nl * 4);
    const floatx4 cb = *reinterpret_cast<const floatx4*>(tc + G2_TC_COLS + 512 + nl * 4);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = pacc[a][b][4 * gq + j] * ai * cs[j] + cb[j];
    if constexpr (EPI == G2_EPI_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gv = gelu_erf(v[j]);
        v[j] = n + j < p.act_ncols ? gv : v[j];
      }
    }
    if constexpr (RES) {
      const floatx4 r = __builtin_bit_cast(floatx4, rvu);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += r[j];
    }
    const bool ok = mok && n < p.N;
    if (ok) ymax = fmaxf(ymax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    const u32x4 pk = {__builtin_bit_cast(unsigned, v[0]), __builtin_bit_cast(unsigned, v[1]),
                      __builtin_bit_cast(unsigned, v[2]), __builtin_bit_cast(unsigned, v[3])};
    if (G2_ABL & 64) asm volatile("" ::"v"(pk));
    else __builtin_amdgcn_raw_buffer_store_b128(pk, rY, (ok && !(G2_ABL & 4)) ? (yrow + (unsigned)n) * 4u : OOB, 0, 0);
  };
  // the previous tile's units of stage kt: each of the 16 unit bodies exists once, run under a uniform predicate
  auto epi_stage = [&](floatx16 (&pacc)[2][2], const G2Tile& ct, int cloc, int kt, const u32x4 (&rv)[4]) {
    auto one = [&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (unit_in(kt, u)) epi_unit(pacc, ct, cloc, uc, rv[u >> 2]);
    };
    one(std::integral_constant<int, 0>{}); one(std::integral_constant<int, 1>{});
    one(std::integral_constant<int, 2>{}); one(std::integral_constant<int, 3>{});
    one(std::integral_constant<int, 4>{}); one(std::integral_constant<int, 5>{});
    one(std::integral_constant<int, 6>{}); one(std::integral_constant<int, 7>{});
    one(std::integral_constant<int, 8>{}); one(std::integral_constant<int, 9>{});
    one(std::integral_constant<int, 10>{}); one(std::integral_constant<int, 11>{});
    one(std::integral_constant<int, 12>{}); one(std::integral_constant<int, 13>{});
    one(std::integral_constant<int, 14>{}); one(std::integral_constant<int, 15>{});
  };
  auto res_stage = [&](u32x4 (&rv)[4], const G2Tile& ct, int kt) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (unit_in(kt, u)) rv[u >> 2] = res_load(ct, u >> 2, u & 3);
  };
  // a tile's column constants, once landed: [winv | bias | scale | shift] -> [winv * scale | bias * scale + shift]
  auto combine_cols = [&](int cloc) {
    if (tid < G2_BN) {
      float* c = reinterpret_cast<float*>(tcb + (cloc % 3) * G2_TC_BYTES + G2_TC_COLS);
      const float sc = p.has_scale ? c[256 + tid] : 1.f;
      const float cb = ((p.has_bias ? c[128 + tid] : 0.f) * sc) + (p.has_shift ? c[384 + tid] : 0.f);
      c[tid] = c[tid] * sc;
      c[128 + tid] = cb;
    }
  };

  // younger vector-memory ops than stage g's DMA at its wait: stage g + 1's 6 pieces, the stores of stage g - 1's
  // epilogue part (issued before those pieces) are older than them but younger than stage g's: 6 + 4
  auto stores_in = [&](int x) { return (x >= nk && x % nk < E2) ? 16 / E2 : 0; };

  u32x4 rv[4];
  auto tile_body = [&](floatx16 (&acc)[2][2], floatx16 (&pacc)[2][2], int tl) {
    const G2Tile pt = g2_tile<MODE>(p, tstart + (tl > 0 ? tl - 1 : 0) * tstep, tiles_n);  // previous tile
    const bool res = RES && tl > 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int g = tl * nk + kt;
#if G2_STAMP
      const unsigned long long t0 = STAMP();
#endif
      const int sy = stores_in(g - 1);
      if (sy == 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(G2_PIECES) : "memory");
      else if (sy == 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(G2_PIECES + 2) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(G2_PIECES + 4) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#if G2_STAMP
      const unsigned long long t1 = STAMP();
      t_wait += t1 - t0;
#endif
      if (kt == 0) combine_cols(tl);  // read by this tile's epilogue, many barriers later
      // the previous tile's epilogue units of this stage: at the stage start on waves 0-3, after the MFMAs on
      // waves 4-7 (the two waves of a SIMD: one stores while the other computes); with a residual all at the start
      // (a residual load waited for after this stage's DMA would wait for the DMA)
      const bool units = tl > 0 && kt < E2;
      const int unit_ph = (wid >= 4 && !RES && !(G2_ABL & 128)) ? 1 : 0;
      if (units && res && kt == 0) res_stage(rv, pt, 0);
      if (kt == 0) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
      }
      // stage g + 2 into the slot every wave finished reading; past the last stage a zero-fill DMA (out-of-range
      // source) into a slot nobody reads again keeps the body branch-free and the piece count fixed
      if (g + 2 < S) prep(g + 2);
      else {
        cur_st = lds + ((g + 2) % G2_STAGES) * G2_STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < G2_PIECES; ++i) cur_off[i] = OOB;
      }
      const char* st = lds + (g % G2_STAGES) * G2_STAGE_BYTES;
      // phase 0 / 1: the previous tile's units of this stage run before the MFMAs on waves 0-3 and after them on
      // waves 4-7 (the two waves of a SIMD: one stores while the other computes); with a residual all before
      if (units && unit_ph == 0) epi_stage(pacc, pt, tl - 1, kt, rv);
      {
#pragma unroll
        for (int s = 0; s < 2; ++s) {  // per 16-deep k-step: 8 fragment reads, 3 groups of 4 MFMAs + 3 DMA pieces
          f16x8 af[2][2], wf[2][2];     // [block][term] (one k-step live at a time: 32 registers)
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            const int r = wm * 64 + a * 32 + r32;
            af[a][0] = *reinterpret_cast<const f16x8*>(st + swz(r, 2 * s + h));
            af[a][1] = *reinterpret_cast<const f16x8*>(st + G2_BM * 64 + swz(r, 2 * s + h));
          }
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int r = wn * 64 + b * 32 + r32;
            wf[b][0] = *reinterpret_cast<const f16x8*>(st + G2_A_BYTES + swz(r, 2 * s + h));
            wf[b][1] = *reinterpret_cast<const f16x8*>(st + G2_A_BYTES + G2_BN * 64 + swz(r, 2 * s + h));
          }
#pragma unroll
          for (int t = 0; t < 3; ++t) {  // term pairs l.h, h.l, h.h
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
              for (int b = 0; b < 2; ++b)
                if (!(G2_ABL & 1))
                  acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[b][t == 1 ? 1 : 0], af[a][t == 0 ? 1 : 0],
                                                                     acc[a][b], 0, 0, 0);
            dma(3 * s + t);
          }
          __builtin_amdgcn_sched_barrier(0);  // keep the next k-step's reads behind these MFMAs (register reuse)
        }
      }
      if (units && unit_ph == 1) epi_stage(pacc, pt, tl - 1, kt, rv);
#if G2_STAMP
      t_mfma += STAMP() - t1;
#endif
      if (res && kt + 1 < E2) res_stage(rv, pt, kt + 1);  // the next stage's residual pieces
    }
  };
  for (int tl = 0; tl < n_my; tl += 2) {
    tile_body(acc0, acc1, tl);
    if (tl + 1 < n_my) tile_body(acc1, acc0, tl + 1);
  }
  // the last tile's epilogue: everything has landed (the last stages' zero-fill DMAs aside)
  {
    const int tl = n_my - 1;
    const G2Tile ct = g2_tile<MODE>(p, tstart + tl * tstep, tiles_n);
    auto last = [&](floatx16 (&acc)[2][2]) {
      u32x4 rl[16];  // all residual pieces first: a load waited for between stores would wait for them too
      if constexpr (RES) {
#pragma unroll
        for (int u = 0; u < 16; ++u) rl[u] = res_load(ct, u >> 2, u & 3);
      }
      auto one = [&](auto uc) { epi_unit(acc, ct, tl, uc, rl[decltype(uc)::value]); };
      one(std::integral_constant<int, 0>{}); one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{}); one(std::integral_constant<int, 3>{});
      one(std::integral_constant<int, 4>{}); one(std::integral_constant<int, 5>{});
      one(std::integral_constant<int, 6>{}); one(std::integral_constant<int, 7>{});
      one(std::integral_constant<int, 8>{}); one(std::integral_constant<int, 9>{});
      one(std::integral_constant<int, 10>{}); one(std::integral_constant<int, 11>{});
      one(std::integral_constant<int, 12>{}); one(std::integral_constant<int, 13>{});
      one(std::integral_constant<int, 14>{}); one(std::integral_constant<int, 15>{});
    };
    if (tl & 1) last(acc1);
    else last(acc0);
  }
#if G2_STAMP
  if (lane == 0) {
    unsigned long long* o = g2_stamp_buf + ((int)blockIdx.x * G2_NW + wid) * 4;
    o[0] = STAMP() - t_begin;
    o[1] = t_wait;
    o[2] = t_mfma;
    o[3] = t_epi;
  }
#endif
  if (p.y_amax) {
    const float m = sfx::wave_max(ymax);
    if (lane == 0)
      atomicMax(p.y_amax + ((int)blockIdx.x * G2_NW + wid) % sfx::kAmaxSub,
                ((unsigned long long)p.y_tag << 32) | __builtin_bit_cast(unsigned, m));
  }
}

// ---- operand pre-split: one wave per row, K padded to Kp with zeros ----------------------------------------
// VEC: rows are 16-byte aligned with K % 4 == 0 and K <= 2048 -- the row stays in registers (8 float4 per lane)
// between its maximum and its split; 8-byte plane stores.
template <bool VEC>
__global__ void __launch_bounds__(256) split_planes_kernel(int rows, int K, int Kp, const float* __restrict__ src,
                                                           long long ld, _Float16* __restrict__ dst, long long plane,
                                                           float* __restrict__ inv) {
  const int row = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = src + (long long)row * ld;
  _Float16* dh = dst + (long long)row * Kp;
  _Float16* dl = dh + plane;
  float m = 0.f;
  if constexpr (VEC) {
    float4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 4 * (lane + 64 * j);
      v[j] = c < K ? *reinterpret_cast<const float4*>(s + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[j].x), fabsf(v[j].y)), fmaxf(fabsf(v[j].z), fabsf(v[j].w))));
    }
    m = sfx::wave_max(m);
    int e = 0;
    if (m > 0.f && m <= 3.4028235e38f) e = min(row_exp(m) + 2, 126);
    const float sc = ldexpf(1.f, e);
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c >= Kp) break;
      const float x[4] = {v[j].x * sc, v[j].y * sc, v[j].z * sc, v[j].w * sc};
      h4 hv, lv;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        hv[i] = (_Float16)x[i];
        lv[i] = (_Float16)(x[i] - (float)hv[i]);
      }
      *reinterpret_cast<h4*>(dh + c) = hv;
      *reinterpret_cast<h4*>(dl + c) = lv;
    }
    if (lane == 0) inv[row] = ldexpf(1.f, -e);
  } else {
    for (int c = lane; c < K; c += 64) m = fmaxf(m, fabsf(s[c]));
    m = sfx::wave_max(m);
    int e = 0;
    if (m > 0.f && m <= 3.4028235e38f) e = min(row_exp(m) + 2, 126);
    const float sc = ldexpf(1.f, e);
    for (int c = lane; c < Kp; c += 64) {
      const float x = c < K ? s[c] * sc : 0.f;
      const _Float16 hv = (_Float16)x;
      dh[c] = hv;
      dl[c] = (_Float16)(x - (float)hv);
    }
    if (lane == 0) inv[row] = ldexpf(1.f, -e);
  }
}

int num_cus2() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

template <int MODE>
void g2_launch(G2Args& a, hipStream_t st) {
  int tiles_m;
  if (MODE == G2_PAIR) {
    tiles_m = 0;
    for (int k = 0; k < a.num_slices; ++k) {
      a.slice_tile_off[k] = tiles_m;
      tiles_m += (a.slice_pair_off[k + 1] - a.slice_pair_off[k] + G2_BM - 1) / G2_BM;
    }
    a.slice_tile_off[a.num_slices] = tiles_m;
  } else {
    tiles_m = (int)sfx::ceil_div(a.M, G2_BM);
  }
  const int tiles_n = (int)sfx::ceil_div(a.N, G2_BN);
  const int total = tiles_m * tiles_n;
  if (total == 0) return;
  const int cus = num_cus2() / 8 * 8;
  const int grid = total <= cus ? total : cus;
  if (MODE == G2_DENSE && a.R) gemm2_kernel<G2_DENSE, G2_EPI_RES><<<grid, 512, 0, st>>>(a, tiles_n, total);
  else if (MODE == G2_DENSE && a.act == ACT_GELU)
    gemm2_kernel<G2_DENSE, G2_EPI_GELU><<<grid, 512, 0, st>>>(a, tiles_n, total);
  else gemm2_kernel<MODE, G2_EPI_AFFINE><<<grid, 512, 0, st>>>(a, tiles_n, total);
}

bool al16(const void* p) { return reinterpret_cast<unsigned long long>(p) % 16 == 0; }

}  // namespace

extern "C" {

#if G2_STAMP
int sfx_gemm2_stamps(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g2_stamp_buf), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif


int sfx_split_planes(int rows, int K, int Kp, const float* x, long long ld, void* dst, long long plane, float* inv,
                     void* stream) {
  SFX_REQUIRE(rows >= 0 && K > 0 && Kp >= K && Kp % 32 == 0 && ld >= K && plane >= (long long)rows * Kp,
              "sfx_split_planes: bad sizes");
  if (rows == 0) return SFX_OK;
  SFX_REQUIRE(x && dst && inv, "sfx_split_planes: null buffer");
  const bool vec = K % 4 == 0 && ld % 4 == 0 && K <= 2048 && reinterpret_cast<unsigned long long>(x) % 16 == 0 &&
                   reinterpret_cast<unsigned long long>(dst) % 8 == 0 && plane % 4 == 0;
  if (vec)
    split_planes_kernel<true><<<sfx::ceil_div(rows, 4), 256, 0, sfx::as_stream(stream)>>>(
        rows, K, Kp, x, ld, static_cast<_Float16*>(dst), plane, inv);
  else
    split_planes_kernel<false><<<sfx::ceil_div(rows, 4), 256, 0, sfx::as_stream(stream)>>>(
        rows, K, Kp, x, ld, static_cast<_Float16*>(dst), plane, inv);
  return sfx::check_launch("sfx_split_planes");
}

// Y[M][N] = epilogue(A' W^T) on pre-split planes (sfx_split_planes; A planes of a_rows rows).  mode 0: A rows m;
// 1: rows gidx[m * gstride] (-1: zero row); epilogue as sfx_linear (bias, BN affine, activation on cols <
// act_ncols, residual R[m]; ridx must be null), optional output bound y_amax / y_tag.  N, ldy, ldr multiples of 4, Kp >= 128,
// 16-byte aligned Y / R / column arrays (sfx_gemm2_ok).
int sfx_gemm2_ok(int N, int Kp, const float* winv, const float* bias, const float* scale, const float* shift,
                 const float* R, long long ldr, const float* Y, long long ldy) {
  return N % 4 == 0 && Kp % 32 == 0 && Kp >= 128 && ldy % 4 == 0 && al16(Y) && al16(winv) && al16(bias) &&
         al16(scale) && al16(shift) && (!R || (ldr % 4 == 0 && al16(R)));
}

int sfx_gemm2(int mode, int M, int N, int Kp, const void* A, long long a_plane, const float* ainv, int a_rows,
              const int* gidx, int gstride, const void* W, long long w_plane, const float* winv, const float* bias,
              const float* scale, const float* shift, int act, int act_ncols, const float* R, long long ldr,
              const int* ridx, float* Y, long long ldy, unsigned long long* y_amax, unsigned y_tag, void* stream) {
  SFX_REQUIRE(mode == 0 || mode == 1, "sfx_gemm2: mode 0 (dense) or 1 (gather)");
  SFX_REQUIRE(M >= 0 && N > 0 && Kp >= 128 && Kp % 32 == 0 && a_rows > 0 && (mode == 1 || a_rows >= M),
              "sfx_gemm2: bad sizes");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(A && ainv && W && winv && Y && (mode == 0 || gidx), "sfx_gemm2: null buffer");
  SFX_REQUIRE(!ridx, "sfx_gemm2: gathered residual rows are not supported (sfx_linear has them)");
  SFX_REQUIRE(!R || mode == 0, "sfx_gemm2: a residual needs mode 0");
  SFX_REQUIRE(act == ACT_NONE || (act == ACT_GELU && mode == 0 && !R),
              "sfx_gemm2: activation GELU (mode 0, no residual) or none");
  SFX_REQUIRE(!R || (!scale && !shift), "sfx_gemm2: a residual goes with bias only");
  SFX_REQUIRE(sfx_gemm2_ok(N, Kp, winv, bias, scale, shift, R, ldr, Y, ldy),
              "sfx_gemm2: N / ldy / ldr must be multiples of 4 and Y / R / column arrays 16-byte aligned");
  SFX_REQUIRE(4 * a_plane < 0x7ffffff0ll && 4 * w_plane < 0x7ffffff0ll && ((long long)M * ldy + N) * 4 < 0x7ffffff0ll &&
                  (mode == 0 || (long long)M * gstride * 4 < 0x7ffffff0ll),
              "sfx_gemm2: operand exceeds the 2 GiB buffer-descriptor range");
  G2Args a{};
  a.M = M; a.N = N; a.Kp = Kp; a.A = static_cast<const _Float16*>(A); a.a_plane = a_plane; a.ainv = ainv;
  a.a_rows = a_rows; a.gidx = gidx; a.gstride = gstride; a.W = static_cast<const _Float16*>(W);
  a.w_plane = w_plane; a.winv = winv;
  a.bias = bias ? bias : winv; a.scale = scale ? scale : winv; a.shift = shift ? shift : winv;
  a.has_bias = bias != nullptr; a.has_scale = scale != nullptr; a.has_shift = shift != nullptr;
  a.act = act; a.act_ncols = act_ncols < 0 ? N : act_ncols;
  a.R = R; a.ldr = ldr; a.Y = Y; a.ldy = ldy; a.y_amax = y_amax; a.y_tag = y_tag;
  hipStream_t st = sfx::as_stream(stream);
  if (mode == 0) g2_launch<G2_DENSE>(a, st);
  else g2_launch<G2_GATHER>(a, st);
  return sfx::check_launch("sfx_gemm2");
}

// SubM pair products on pre-split planes: the 26 non-centre offsets' pair lists (sfx_subm_pairs, pair_off_host =
// the 28 offsets) as one flat tile list; W planes [27][N][Kp] (27 * N split rows), winv [27][N]; the product of
// pair p is stored at row p of Y (sfx_cpe_residual_ln_pairs sums a row's pairs).
int sfx_gemm2_pairs(int N, int Kp, const void* A, long long a_plane, const float* ainv, int a_rows,
                    const int* pair_in, const int* pair_off_host, const void* W, long long w_plane, const float* winv,
                    float* Y, long long ldy, void* stream) {
  SFX_REQUIRE(N > 0 && Kp >= 128 && Kp % 32 == 0 && a_rows > 0 && pair_off_host, "sfx_gemm2_pairs: bad sizes");
  if (pair_off_host[27] == 0) return SFX_OK;
  SFX_REQUIRE(A && ainv && pair_in && W && winv && Y, "sfx_gemm2_pairs: null buffer");
  SFX_REQUIRE(sfx_gemm2_ok(N, Kp, winv, nullptr, nullptr, nullptr, nullptr, 0, Y, ldy) && (27ll * N) % 4 == 0,
              "sfx_gemm2_pairs: N / ldy must be multiples of 4 and Y / winv 16-byte aligned");
  SFX_REQUIRE(4 * a_plane < 0x7ffffff0ll && 4 * w_plane < 0x7ffffff0ll && w_plane >= 27ll * N * Kp &&
                  ((long long)pair_off_host[27] * ldy) * 4 < 0x7ffffff0ll,
              "sfx_gemm2_pairs: operand exceeds the 2 GiB buffer-descriptor range");
  G2Args a{};
  a.N = N; a.Kp = Kp; a.A = static_cast<const _Float16*>(A); a.a_plane = a_plane; a.ainv = ainv; a.a_rows = a_rows;
  a.gidx = pair_in; a.gstride = 1; a.W = static_cast<const _Float16*>(W); a.w_plane = w_plane; a.winv = winv;
  a.bias = a.scale = a.shift = winv;
  a.act = 0; a.act_ncols = N; a.Y = Y; a.ldy = ldy;
  a.num_slices = 27;
  for (int k = 0; k <= 27; ++k) a.slice_pair_off[k] = pair_off_host[k];
  a.M = pair_off_host[27];
  g2_launch<G2_PAIR>(a, sfx::as_stream(stream));
  return sfx::check_launch("sfx_gemm2_pairs");
}

}  // extern "C"
