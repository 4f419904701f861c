// Host side of the fp32-accurate MFMA GEMM family: tile tables, operand maxima, dispatch and the C-ABI entries
// (the kernel template: gemm_kernel.h, instantiated per operand mode in gemm_k*.hip).
#include <climits>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "gemm_common.h"


namespace {

using namespace sfxg;

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline bool fits(long long rows, long long ld) { return rows * ld * 4 + 64 < (long long)OOB; }

// Tile shapes.  The choice minimises (rounds of per-CU slots) x (tile area / relative efficiency): with
// K = 64..2048 and M = 15k..100k every layer is a few rounds of tiles, so wave quantisation and N-padding
// (N = 96, 288 on the C=96 stages) decide more than peak per-tile efficiency.  The eight-wave tiles exist
// only with split operands.
struct TileCfg {
  int bm, bn, nw;
  float eff;
};
constexpr TileCfg kCfgs[] = {{128, 128, 4, 1.0f}, {128, 96, 4, 0.95f}, {128, 64, 4, 0.8f}, {64, 128, 4, 0.95f},
                             {64, 64, 4, 0.8f},   {256, 128, 8, 1.05f}, {128, 256, 8, 1.05f}};  // eff: tools/gemm_calls.py sweeps
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

// Operand precision: the 3-term bf16 split (fp32-accurate, see gemm_kernel) from K >= split_min_k
// (SFX_GEMM_SPLIT_MINK; default 64), exact fp32 MFMA below it or with SFX_GEMM_PREC=fp32.
// Operand precision of a launch (GemmArgs::split): exact fp32 MFMA below K = 64 (SFX_GEMM_SPLIT_MINK) or with
// SFX_GEMM_PREC=fp32; otherwise split operands, fp16x2 (default) or bf16x3 (SFX_GEMM_PREC=bf16x3).  Both split
// forms are as accurate as fp32 arithmetic; fp16x2 needs half the MFMAs and LDS images of bf16x3.
// library precision mode (sfx_set_precision): 0 fp32-accurate (default), 1 reference precision (autocast class);
// per host thread, so a launch from another thread (an eval pass beside a Trainer inside its amp region) keeps
// its own mode
thread_local int g_prec = 0;

int split_mode(int K) {
  static int min_k = -2, mode = 2;
  if (min_k == -2) {
    const char* e = getenv("SFX_GEMM_PREC");
    const char* m = getenv("SFX_GEMM_SPLIT_MINK");
    const bool f32 = e && !strcmp(e, "fp32");
    mode = (e && !strcmp(e, "bf16x3")) ? 3 : 2;
    min_k = f32 ? -1 : ((m && *m) ? atoi(m) : 64);
  }
  return (min_k >= 0 && K >= min_k) ? mode : 0;
}

// ---- fp16x2 operand maxima -------------------------------------------------------------------------------
// max |x| over a GEMM operand, atomically max-ed into a slot as (tag << 32 | float bits): a launch's larger tag
// supersedes whatever an earlier launch left, so slots need no clearing.  A' is read as the GEMM reads it
// (dense rows, or gathered rows of S segments of Kseg columns; `groups` copies at a group stride).
struct AmaxJob {
  const float* base;
  long long ld, group_stride;
  int rows, cols, groups;  // cols per (gathered) segment
  const int* gidx;         // [rows][gstride] gather index (first S used) or null
  int gstride, S;
};

__global__ void __launch_bounds__(256) amax_kernel(AmaxJob j0, AmaxJob j1, unsigned long long* slot0,
                                                   unsigned long long* slot1, unsigned tag0, unsigned tag1) {
  const AmaxJob j = blockIdx.y == 0 ? j0 : j1;
  // one wave per (group, row, segment): lanes sweep the row's columns, 16 B per lane where aligned
  const int per_group = j.rows * j.S;
  const int segs = j.groups * per_group;
  const int wave = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), nwaves = (int)gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  const bool vec = (j.cols % 4 == 0) && (j.ld % 4 == 0) && (j.group_stride % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(j.base) & 15) == 0);
  float m = 0.f;
  const bool flat = !j.gidx && j.ld == j.cols && (j.groups == 1 || j.group_stride == (long long)j.rows * j.ld);
  if (flat && vec) {  // one contiguous array (the common case): 4 independent 16-byte loads in flight per lane
    const long long n4 = (long long)segs * j.cols / 4;
    const float4* q = reinterpret_cast<const float4*>(j.base);
    const long long stride = (long long)gridDim.x * 256;
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    for (; i + 7 * stride < n4; i += 8 * stride) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = q[i + u * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    for (; i < n4; i += stride) {
      const float4 v = q[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  }
  for (int sg = flat && vec ? segs : __builtin_amdgcn_readfirstlane(wave); sg < segs; sg += nwaves) {
    const int g = sg / per_group;
    const int rs = sg - g * per_group;
    const int r0 = j.S == 1 ? rs : rs / j.S, seg = rs - r0 * j.S;
    const long long row = j.gidx ? (long long)j.gidx[(long long)r0 * j.gstride + seg] : r0;
    if (row < 0) continue;
    const float* q = j.base + (long long)g * j.group_stride + row * j.ld;
    if (vec) {
      for (int c = lane * 4; c < j.cols; c += 256) {
        const float4 v = *reinterpret_cast<const float4*>(q + c);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
    } else {
      for (int c = lane; c < j.cols; c += 64) m = fmaxf(m, fabsf(q[c]));
    }
  }
  __shared__ float wmax[4];
  // one atomic per workgroup, spread over the 64 sub-slots (same-address atomics serialise)
  sfx::publish_amax(m, blockIdx.y == 0 ? slot0 : slot1, blockIdx.y == 0 ? tag0 : tag1, wmax);
}

// amax slots of the library's own maxima passes: a per-device ring; stream order makes a slot's producer
// (amax_kernel) and consumer (the GEMM) adjacent, the ring keeps launches queued on other streams apart
unsigned long long* amax_slot() {
  constexpr int kSlots = 2048;
  static unsigned long long* bufs[64] = {};
  static unsigned next[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!bufs[dev]) {
    if (hipMalloc(&bufs[dev], sizeof(unsigned long long) * sfx::kAmaxSub * kSlots) != hipSuccess) return nullptr;
    (void)hipMemset(bufs[dev], 0, sizeof(unsigned long long) * sfx::kAmaxSub * kSlots);
  }
  return bufs[dev] + sfx::kAmaxSub * (next[dev]++ % kSlots);
}

unsigned next_amax_tag() {
  static unsigned tag = 0;
  if (++tag == 0) ++tag;  // 0 never matches (fresh slots hold zeros)
  return tag;
}

int amax_blocks(const AmaxJob& j) {  // >= 32 KB of operand per wave, at most 2 workgroups per CU
  const long long bytes = (long long)j.groups * j.rows * j.S * j.cols * 4;
  const long long b = (bytes + 4 * 32768 - 1) / (4 * 32768);
  const long long cap = 2ll * num_cus();
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

// queue the maxima passes an fp16x2 launch lacks (A' and / or W); false on slot-allocation failure
bool prepare_amax(GemmArgs& a, const AmaxJob& ja, const AmaxJob& jw, hipStream_t st) {
  const bool need_a = !a.a_amax, need_w = !a.w_amax;
  if (!need_a && !need_w) return true;
  unsigned long long* sa = need_a ? amax_slot() : nullptr;
  unsigned long long* sw = need_w ? amax_slot() : nullptr;
  if ((need_a && !sa) || (need_w && !sw)) return false;
  const unsigned ta = need_a ? next_amax_tag() : 0, tw = need_w ? next_amax_tag() : 0;
  const AmaxJob& j0 = need_a ? ja : jw;
  const int bx = (need_a && need_w) ? (amax_blocks(ja) > amax_blocks(jw) ? amax_blocks(ja) : amax_blocks(jw))
                                    : amax_blocks(j0);
  amax_kernel<<<dim3(bx, need_a && need_w ? 2 : 1), 256, 0, st>>>(j0, jw, need_a ? sa : sw, sw, need_a ? ta : tw,
                                                                  tw);
  if (need_a) { a.a_amax = sa; a.a_tag = ta; }
  if (need_w) { a.w_amax = sw; a.w_tag = tw; }
  return true;
}

// the operand jobs of a GemmArgs (non-pair launches; pair launches get the maxima from their caller)
void gemm_amax_jobs(const GemmArgs& a, int groups, AmaxJob& ja, AmaxJob& jw) {
  ja = AmaxJob{a.A, a.lda, a.gA, a.M, a.gidx ? a.Kseg : a.K, groups, a.gidx, a.gstride, a.gidx ? a.S : 1};
  jw = AmaxJob{a.W, a.ldw, a.gW, a.N, a.K, groups, nullptr, 0, 1};
}

// Measured per-launch best (tile configuration, Stream-K) for the config-B (and config-E) refine's dense linears
// under fp16x2 operands (tools/gemm_tune.py; profiles/r01_gemm_tune_f16x2.jsonl, re-swept with the per-row scales in
// profiles/r02_gemm_tune.jsonl) where it beats the cost model by > 2 us;
// applied when N and K match and M is within 0.8-1.25x of the tuned M (stage point counts vary per scene).
struct TunedLaunch {
  int M, N, K, cfg, sk;
};
constexpr TunedLaunch kTuned[] = {
    {100000, 64, 23, 2, 0},
    {100000, 256, 64, 1, 1},
    {90434, 128, 96, 3, 1},
    {70349, 384, 128, 1, 0},
    {70349, 128, 128, 3, 0},
    {70349, 512, 128, 3, 1},
    {70349, 128, 512, 3, 0},
    {70349, 256, 128, 3, 1},
    {37759, 768, 256, 6, 0},
    {37759, 256, 256, 1, 1},
    {37759, 256, 1024, 1, 0},
    {37759, 512, 256, 6, 1},
    {14764, 1536, 512, 6, 0},
    {14764, 2048, 512, 6, 1},
    {14764, 512, 2048, 6, 0},
    {100000, 768, 120, 6, 0},
    {37759, 1024, 256, 6, 1},
    {14764, 512, 512, 6, 0},
    {70349, 96, 128, 1, 0},
    {100000, 384, 96, 1, 1},
    // config E (500k SH3) stages: profiles/r02_gemm_tune_configE.jsonl
    {500000, 256, 64, 1, 1},
    {329874, 384, 96, 1, 1},
    {329874, 128, 96, 3, 0},
    {167925, 128, 128, 3, 0},
    {167925, 512, 128, 6, 1},
    {167925, 128, 512, 5, 0},
    {167925, 256, 128, 6, 1},
    {66844, 768, 256, 6, 0},
    {66844, 1024, 256, 6, 0},
    {66844, 256, 1024, 6, 1},
    {66844, 512, 256, 6, 1},
    {31270, 1536, 512, 6, 0},
    {31270, 512, 512, 6, 0},
    {31270, 2048, 512, 6, 0},
    {31270, 512, 2048, 5, 0},
    {31270, 256, 512, 6, 0},
    {66844, 128, 256, 3, 1},
    {500000, 384, 96, 1, 0},
    {500000, 768, 156, 6, 1},
    {500000, 59, 768, 2, 0}};

// The same for the SubM conv launches of config B's stages (sfx_subm_conv: n, Cout, Cin -> the tile shape /
// Stream-K of its centre and pair launches; re-swept for the per-pair-store form,
// profiles/r02_gemm_tune_conv_partials.jsonl -- Stream-K only applies to the atomic form; round 6 re-sweep with the
// centre offset in the eval pair lists, profiles/r06_gemm_tune.jsonl: stage 2 -> 128x128 tiles (86 vs 103 us),
// stage 0 -> 128x96 (37 vs 43 us))
constexpr TunedLaunch kTunedConv[] = {
    {90434, 96, 96, 1, 1},
    {70349, 128, 128, 0, 0},
    {100000, 64, 64, 1, 0},
    {37759, 256, 256, 6, 1},
    {14764, 512, 512, 6, 0},
    {100000, 96, 96, 1, 0},
    // config E (500k SH3) stages: profiles/r02_gemm_tune_configE.jsonl
    {500000, 64, 64, 2, 1},
    {329874, 96, 96, 1, 0},
    {167925, 128, 128, 5, 0},
    {66844, 256, 256, 6, 0},
    {31270, 512, 512, 6, 0},
    {500000, 96, 96, 1, 1}};

// tuning / test hooks: SFX_GEMM_CFG=<index into kCfgs>, SFX_GEMM_SK=0|1, or sfx_gemm_force_config()
int forced = -2, forced_sk = -2;
void read_force_env() {
  if (forced != -2) return;
  const char* e = getenv("SFX_GEMM_CFG");
  forced = (e && *e) ? atoi(e) : -1;
  if (forced >= kNumCfgs) forced = -1;
  const char* k = getenv("SFX_GEMM_SK");
  forced_sk = (k && *k) ? atoi(k) : -1;
}

// -> configuration index; sets a.sk when the Stream-K split of the same tile shape is cheaper.
int pick_cfg(GemmArgs& a, int groups, bool vec) {
  read_force_env();
  const int nk = (int)sfx::ceil_div(a.K, BK);
  const bool split = a.split != 0;
  // eight-wave tiles exist only with split operands
  const int force = (forced >= 0 && !(kCfgs[forced].nw == 8 && !split)) ? forced : -1;
  // Stream-K needs a linear epilogue that can be split into atomically added pieces
  // (measured: the memset + atomic partial epilogues only pay off on long K; pair mode needs no memset)
  const bool sk_ok = groups == 1 && nk >= (a.pair_mode ? 8 : 16) && a.act == ACT_NONE && !a.Ypre && !a.out_rows &&
                     !a.pair_store &&
                     !a.y_amax &&
                     !(a.R && a.R == a.Y) && a.M > 0 && forced_sk != 0;
  const double sk_overhead = a.pair_mode ? 2.5 : 4.0;  // slab-equivalents: partial epilogues (+ memset)
  if (force < 0 && forced_sk < 0 && a.tuned > 0 && !((kCfgs[a.tuned - 1].nw == 8) && !split)) {
    const int c = a.tuned - 1;
    a.sk = (a.tuned_sk && sk_ok && kCfgs[c].bm >= 128) ? 1 : 0;
    tiles_m_of(a, kCfgs[c].bm);
    return c;
  }
  if (force < 0 && forced_sk < 0 && !a.pair_mode && !a.gidx && groups == 1) {
    for (const TunedLaunch& t : kTuned) {
      if (t.N == a.N && t.K == a.K && 5ll * a.M >= 4ll * t.M && 4ll * a.M <= 5ll * t.M &&
          !((kCfgs[t.cfg].nw == 8) && !split)) {
        a.sk = (t.sk && sk_ok && kCfgs[t.cfg].bm >= 128) ? 1 : 0;
        tiles_m_of(a, kCfgs[t.cfg].bm);
        return t.cfg;
      }
    }
  }
  int best = 0;
  bool best_sk = false;
  double best_cost = 1e300;
  for (int c = 0; c < kNumCfgs; ++c) {
    if (force >= 0 && c != force) continue;
    if (kCfgs[c].nw == 8 && !split) continue;
    const int per_cu = kCfgs[c].nw == 4 ? kPerCu4 : kPerCu8;
    const long long slots = (long long)per_cu * num_cus() / groups;
    // tile area per unit of CU throughput (a resident tile has 1 / per_cu of its CU)
    const double area = (double)kCfgs[c].bm * kCfgs[c].bn / kCfgs[c].eff * per_cu / 2;
    const long long tiles = (long long)tiles_m_of(a, kCfgs[c].bm) * sfx::ceil_div(a.N, kCfgs[c].bn) * groups;
    const long long rounds = (tiles + slots - 1) / slots;
    // cost in slab-area units: K slabs + ~1 slab-equivalent of epilogue per tile
    double cost = (double)rounds * (nk + 1) * area;
    bool sk = false;
    if (sk_ok && kCfgs[c].bm >= 128) {  // Stream-K on the 128-row shapes: ~1.5 extra slab-equivalents (2 partial epilogues)
      const double sk_cost = ((double)((tiles * nk + slots - 1) / slots) + sk_overhead) * area;
      if (sk_cost < cost || forced_sk == 1) {
        cost = sk_cost;
        sk = true;
      }
    }
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
      best_sk = sk;
    }
  }
  a.sk = best_sk ? 1 : 0;
  tiles_m_of(a, kCfgs[best].bm);  // pair mode: slice_tile_off for the chosen shape
  return best;
}

template <int MODE>
void dispatch_mode(GemmArgs a, int groups, bool vec, hipStream_t st) {
  const int cfg = pick_cfg(a, groups, vec);
  const bool w8 = kCfgs[cfg].nw == 8;
  switch (MODE) {
    case MODE_DENSE: (w8 ? launch_m0_w8 : launch_m0_w4)(cfg, a, groups, vec, st); break;
    case MODE_GATHER1: (w8 ? launch_m1_w8 : launch_m1_w4)(cfg, a, groups, vec, st); break;
    default: (w8 ? launch_m3_w8 : launch_m3_w4)(cfg, a, groups, vec, st); break;
  }
}

void dispatch(const GemmArgs& a0, int groups, bool vec, hipStream_t st) {
  GemmArgs a = a0;
  static const int dbg = getenv("SFX_GEMM_DEBUG") ? atoi(getenv("SFX_GEMM_DEBUG")) : 0;  // timing ablations
  a.dbg = dbg;
  a.split = vec ? split_mode(a.K) : 0;
  // fp16x2 needs the pre-split W (per-row scales of A' are chosen in the kernel); without one the launch runs the
  // range-safe bf16x3 form.
  if (a.split == 2 && !a.Wsp) a.split = 3;
  if (a.split == 2 && g_prec == 1) a.split = 1;  // reference-precision mode: single fp16 term
  if (a.pair_mode)
    dispatch_mode<MODE_PAIR>(a, groups, vec, st);
  else if (!a.gidx)
    dispatch_mode<MODE_DENSE>(a, groups, vec, st);
  else if (a.S == 1)
    dispatch_mode<MODE_GATHER1>(a, groups, vec, st);
  else
    launch_m2_w4(3, a, groups, vec, st);  // multi-segment gather (64 x 128 tiles): test/reference path only
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

// ---- weight gradient: dW[N, K] += dY[M, N]^T X[M, K] (reduction over the point rows) ----------------
// Output tiles are few (N x K of one layer), the reduction long (M = 10^4..10^5 rows): the M range is
// split over grid.y and every split adds its partial tile with float atomics.  Operands are read
// row-major (n / k contiguous) and transposed into the MFMA layout on the LDS store.
constexpr int WG_TILE = 64;

__global__ void __launch_bounds__(THREADS) wgrad_kernel(int M, int N, int K, const float* __restrict__ dY,
                                                        long long ldy, const float* __restrict__ X, long long ldx,
                                                        float* __restrict__ dW, long long ldw, int chunk,
                                                        float* __restrict__ db) {
  __shared__ __attribute__((aligned(16))) float sA[WG_TILE * LDS_STRIDE];
  __shared__ __attribute__((aligned(16))) float sB[WG_TILE * LDS_STRIDE];
  const int tiles_k = (K + WG_TILE - 1) / WG_TILE;
  const int n0 = (blockIdx.x / tiles_k) * WG_TILE, k0 = (blockIdx.x % tiles_k) * WG_TILE;
  const int m_begin = blockIdx.y * chunk;
  const int m_end = min(M, m_begin + chunk);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int lrow = tid & 31, lc4 = (tid >> 5) * 4;  // staging: slab row, 4-column group (+32 for the 2nd)
  const __amdgpu_buffer_rsrc_t rY = rsrc(dY);
  const __amdgpu_buffer_rsrc_t rX = rsrc(X);
  const unsigned ldy32 = (unsigned)ldy, ldx32 = (unsigned)ldx;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // bias gradient (db = column sums of dY) rides along in the k-tile-0 workgroups: thread tid < 64 owns
  // column n0 + tid of the staged dY slab
  const bool do_db = db != nullptr && k0 == 0;
  float dbs = 0.f;
  for (int m0 = m_begin; m0 < m_end; m0 += BK) {
    const int m = m0 + lrow;
    const bool mok = m < m_end;
    float4 ya[2], xb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = n0 + lc4 + 32 * i, k = k0 + lc4 + 32 * i;
      ya[i] = bload4(rY, (mok && n < N) ? ((unsigned)m * ldy32 + (unsigned)n) * 4u : OOB);
      xb[i] = bload4(rX, (mok && k < K) ? ((unsigned)m * ldx32 + (unsigned)k) * 4u : OOB);
    }
    __syncthreads();  // previous slab fully consumed
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = lc4 + 32 * i;
      sA[(c + 0) * LDS_STRIDE + lrow] = ya[i].x;
      sA[(c + 1) * LDS_STRIDE + lrow] = ya[i].y;
      sA[(c + 2) * LDS_STRIDE + lrow] = ya[i].z;
      sA[(c + 3) * LDS_STRIDE + lrow] = ya[i].w;
      sB[(c + 0) * LDS_STRIDE + lrow] = xb[i].x;
      sB[(c + 1) * LDS_STRIDE + lrow] = xb[i].y;
      sB[(c + 2) * LDS_STRIDE + lrow] = xb[i].z;
      sB[(c + 3) * LDS_STRIDE + lrow] = xb[i].w;
    }
    __syncthreads();
    if (do_db && tid < WG_TILE) {
#pragma unroll
      for (int j = 0; j < BK; j += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&sA[tid * LDS_STRIDE + j]);
        dbs += (v.x + v.y) + (v.z + v.w);
      }
    }
    const float* a_lds = &sA[(wm * 32 + l32) * LDS_STRIDE + h * 16];
    const float* b_lds = &sB[(wn * 32 + l32) * LDS_STRIDE + h * 16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 af = *reinterpret_cast<const float4*>(a_lds + 4 * c);
      const float4 bf = *reinterpret_cast<const float4*>(b_lds + 4 * c);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.x, bf.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.y, bf.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.z, bf.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af.w, bf.w, acc, 0, 0, 0);
    }
  }
  if (do_db && tid < WG_TILE && n0 + tid < N) atomicAdd(&db[n0 + tid], dbs);
  const __amdgpu_buffer_rsrc_t rW = rsrc(dW);
  const int k = k0 + wn * 32 + l32;
  const unsigned ldw32 = (unsigned)ldw;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = n0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(acc[r], rW, (n < N && k < K) ? ((unsigned)n * ldw32 + (unsigned)k) * 4u
                                                                                 : OOB, 0, 0);
  }
}

// bf16x3 form (default): the same reduction on v_mfma_f32_32x32x16_bf16 with both operands as three bf16 terms
// (sfx::split3, the six leading term products: fp32 accuracy, no scaling) and 128 x 128 output tiles -- at 64 x 64
// every dY column block is re-read K/64 times and every X column block N/64 times, which bound the exact kernel
// (the (768, 256, 37759) qkv gradient moved ~0.93 GB for 0.15 GB of operands).  Staging: a thread loads 8 points
// x 4 columns (coalesced row segments) and writes, per column and term, the 8 points as one 16-byte chunk of a
// [column][32 points] bf16 image with 64-byte rows (chunk c of row r at c ^ ((r >> 2) & 3)), i.e. already in the
// MFMA fragment order (lane = output row / column, 8 consecutive points per half-wave); the next slab's loads
// are in flight while the current one is multiplied.
constexpr int WG2_T = 128;  // output tile rows (n) and columns (k)
constexpr int WG2_PLANE = WG2_T * 64;  // bytes of one term image

// NQ = 2 (reference-precision mode): the two leading terms and three products t0t0, t0t1, t1t0 (16-bit
// significands, still finer than the reference autocast's fp16 operands).
template <int NQ>
__global__ void __launch_bounds__(256, 2) wgrad2_kernel(int M, int N, int K, const float* __restrict__ dY,
                                                        long long ldy, const float* __restrict__ X, long long ldx,
                                                        float* __restrict__ dW, long long ldw, int chunk,
                                                        float* __restrict__ db) {
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(16))) char img[2 * 3 * WG2_PLANE];  // [dY, X][term][128 rows][64 B]
  const int tiles_k = (K + WG2_T - 1) / WG2_T;
  const int n0 = (blockIdx.x / tiles_k) * WG2_T, k0 = (blockIdx.x % tiles_k) * WG2_T;
  const int m_begin = blockIdx.y * chunk;
  const int m_end = min(M, m_begin + chunk);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int wn = wid & 1, wk = wid >> 1;  // wave sub-tile: rows wn*64.., columns wk*64..
  // staging role: operand op (0 dY, 1 X), column group c4 (4 columns), point group mg (8 points)
  const int op = tid >> 7, c4 = tid & 31, mg = (tid >> 5) & 3;
  const int col = (op ? k0 : n0) + 4 * c4;
  const bool col_ok = col < (op ? K : N);
  const __amdgpu_buffer_rsrc_t rS = rsrc(op ? X : dY);
  const unsigned ld32 = (unsigned)(op ? ldx : ldy);
  auto chunk_off = [](int r, int c) -> int { return r * 64 + (((c ^ (r >> 2)) & 3) << 4); };
  const bool do_db = db != nullptr && k0 == 0 && op == 0;
  float dbs[4] = {0.f, 0.f, 0.f, 0.f};

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float4 v[8];
  auto load = [&](int m0) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int m = m0 + 8 * mg + r;
      v[r] = bload4(rS, (m < m_end && col_ok) ? ((unsigned)m * ld32 + (unsigned)col) * 4u : OOB);
    }
  };
  load(m_begin);
  for (int m0 = m_begin; m0 < m_end; m0 += BK) {
    __syncthreads();  // the previous slab's fragments have been read
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 lo = make_float4(((const float*)&v[0])[j], ((const float*)&v[1])[j], ((const float*)&v[2])[j],
                                    ((const float*)&v[3])[j]);
      const float4 hi = make_float4(((const float*)&v[4])[j], ((const float*)&v[5])[j], ((const float*)&v[6])[j],
                                    ((const float*)&v[7])[j]);
      if (do_db) dbs[j] += ((lo.x + lo.y) + (lo.z + lo.w)) + ((hi.x + hi.y) + (hi.z + hi.w));
      uint2 t0[3], t1[3];
      sfx::split3(lo, t0);
      sfx::split3(hi, t1);
      const int row = 4 * c4 + j;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        *reinterpret_cast<uint4*>(img + (op * 3 + q) * WG2_PLANE + chunk_off(row, mg)) =
            make_uint4(t0[q].x, t0[q].y, t1[q].x, t1[q].y);
    }
    __syncthreads();
    if (m0 + BK < m_end) load(m0 + BK);  // next slab in flight during the products
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // 16-point steps
      bf16x8 af[2][3], bf[2][3];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          af[i][q] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                    img + q * WG2_PLANE + chunk_off(wn * 64 + i * 32 + l32, 2 * s + h)));
          bf[i][q] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                                    img + (3 + q) * WG2_PLANE + chunk_off(wk * 64 + i * 32 + l32, 2 * s + h)));
        }
      constexpr int QA[6] = {2, 1, 0, 1, 0, 0}, QB[6] = {0, 1, 2, 0, 1, 0};  // smallest products first
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int p = NQ == 3 ? 0 : 3; p < 6; ++p)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][QA[p]], bf[j][QB[p]], acc[i][j], 0, 0, 0);
    }
  }
  if (do_db) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (col + j < N) atomicAdd(&db[col + j], dbs[j]);
  }
  const __amdgpu_buffer_rsrc_t rW = rsrc(dW);
  const unsigned ldw32 = (unsigned)ldw;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = k0 + wk * 64 + j * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(
            acc[i][j][r], rW, (n < N && k < K) ? ((unsigned)n * ldw32 + (unsigned)k) * 4u : OOB, 0, 0);
      }
    }
}

// dst[c][r] = src[r][c]
__global__ void __launch_bounds__(256) transpose_kernel(int rows, int cols, const float* __restrict__ src,
                                                        long long lds, float* __restrict__ dst, long long ldd) {
  __shared__ float t[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < rows && c < cols) ? src[(long long)r * lds + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[(long long)c * ldd + r] = t[tx][i];
  }
}


// centre-offset pair lists for the SubM backward: gather row i of dY, add into row nbr[i][13] of dX
__global__ void centre_pairs_kernel(int n, const int* __restrict__ nbr, int* __restrict__ gather,
                                    int* __restrict__ scatter) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  gather[i] = i;
  scatter[i] = nbr[(long long)i * 27 + 13];
}

}  // namespace

extern "C" {

// See include/sfx.h for the contract.
int sfx_gemm_force_config(int cfg, int stream_k) {
  SFX_REQUIRE(cfg >= -1 && cfg < kNumCfgs && stream_k >= -1 && stream_k <= 1, "sfx_gemm_force_config: bad values");
  read_force_env();  // so the environment defaults are not applied over the hook later
  forced = cfg;
  forced_sk = stream_k;
  return SFX_OK;
}

int sfx_weight_split(int rows, int cols, const float* w, long long ld, float* w_split, float* w_inv, void* stream) {
  SFX_REQUIRE(rows >= 0 && cols > 0 && cols % 4 == 0 && ld >= cols && ld % 4 == 0,
              "sfx_weight_split: bad sizes (cols and ld must be multiples of 4)");
  if (rows == 0) return SFX_OK;
  SFX_REQUIRE(w && w_split && w_inv, "sfx_weight_split: null buffer");
  SFX_REQUIRE((reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(w_split) & 15) == 0,
              "sfx_weight_split: buffers must be 16-byte aligned");
  weight_split_kernel<<<sfx::ceil_div(rows, 4), 256, 0, sfx::as_stream(stream)>>>(rows, cols, w, ld, w_split, w_inv);
  return sfx::check_launch("sfx_weight_split");
}

int sfx_amax_f32(int rows, int cols, const float* x, long long ld, unsigned long long* slot, unsigned tag,
                 void* stream) {
  SFX_REQUIRE(rows >= 0 && cols >= 0 && ld >= cols, "sfx_amax_f32: bad sizes");
  SFX_REQUIRE(slot && tag != 0, "sfx_amax_f32: null slot or tag 0");
  SFX_REQUIRE(rows == 0 || cols == 0 || x, "sfx_amax_f32: null buffer");
  const AmaxJob j{x, ld, 0, rows, cols, 1, nullptr, 0, 1};
  amax_kernel<<<dim3(amax_blocks(j), 1), 256, 0, sfx::as_stream(stream)>>>(j, j, slot, slot, tag, tag);
  return sfx::check_launch("sfx_amax_f32");
}

int sfx_linear(int M, int N, int K, const float* A, long long lda, const int* gather_idx, int num_segments,
               const float* W, long long ldw, const float* bias, const float* scale, const float* shift, int act,
               int act_ncols, const float* R, long long ldr, const int* residual_idx, float* Y, long long ldy,
               float* Ypre, long long ldypre, int groups, long long group_stride_A, long long group_stride_W,
               long long group_stride_bias, long long group_stride_Y, const int* out_row_idx, const float* rowscale,
               int pre_before_act, const unsigned long long* a_amax, unsigned a_tag,
               const unsigned long long* w_amax, unsigned w_tag, unsigned long long* y_amax, unsigned y_tag,
               const float* w_split, const float* w_inv, void* stream) {
  SFX_REQUIRE(M >= 0 && N > 0 && K > 0, "sfx_linear: bad sizes M=%d N=%d K=%d", M, N, K);
  SFX_REQUIRE(act >= 0 && act <= 3, "sfx_linear: bad activation %d", act);
  SFX_REQUIRE(groups >= 1, "sfx_linear: groups < 1");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(A && W && Y, "sfx_linear: null buffer");
  const int S = gather_idx ? num_segments : 1;
  SFX_REQUIRE(!gather_idx || (S >= 1 && K % S == 0), "sfx_linear: K must be a multiple of num_segments");
  const int Kseg = K / S;
  SFX_REQUIRE(!gather_idx || Kseg % 4 == 0, "sfx_linear: gathered segment width must be a multiple of 4");
  SFX_REQUIRE(ldw >= K && (gather_idx || lda >= K) && ldy >= N, "sfx_linear: leading dimension too small");
  SFX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), "sfx_linear: scale and shift go together");
  SFX_REQUIRE((gather_idx || fits(M, lda)) && fits(M, ldy) && fits(N, ldw) && (!R || residual_idx || fits(M, ldr)) &&
                  (!Ypre || fits(M, ldypre)),
              "sfx_linear: operand exceeds the 2 GiB buffer-descriptor range");
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.gidx = gather_idx; a.S = S; a.Kseg = Kseg; a.gstride = S;
  a.W = W; a.ldw = ldw; a.bias = bias; a.scale = scale; a.shift = shift; a.act = act;
  a.act_ncols = act_ncols < 0 ? N : act_ncols; a.R = R; a.ldr = ldr; a.ridx = residual_idx; a.Y = Y; a.ldy = ldy;
  a.Ypre = Ypre; a.ldypre = ldypre; a.gA = group_stride_A; a.gW = group_stride_W; a.gB = group_stride_bias;
  a.gY = group_stride_Y; a.out_rows = out_row_idx; a.rowscale = rowscale; a.pre_before_act = pre_before_act;
  a.a_amax = a_amax; a.a_tag = a_tag; a.w_amax = w_amax; a.w_tag = w_tag; a.y_amax = y_amax; a.y_tag = y_tag;
  const bool vec = (K % 4 == 0) && (lda % 4 == 0) && (ldw % 4 == 0) && aligned16(A) && aligned16(W) &&
                   (group_stride_A % 4 == 0) && (group_stride_W % 4 == 0);
  SFX_REQUIRE(!w_split == !w_inv, "sfx_linear: w_split and w_inv go together");
  if (w_split && vec && aligned16(w_split)) {  // split layout: contiguous [groups * N][K], group stride N * K
    SFX_REQUIRE(groups == 1 || group_stride_W == (long long)N * K, "sfx_linear: w_split needs contiguous groups");
    a.Wsp = w_split; a.ldws = K; a.winv = w_inv; a.gWinv = N;
  }
  dispatch(a, groups, vec, sfx::as_stream(stream));
  return sfx::check_launch("sfx_linear");
}

// SubMConv3d, offset-major sparse form.  out = bias + x[nbr[:,13]] W_13^T (dense centre launch, plain
// stores), then one launch over the 26 other offsets' pair lists (pairs from sfx_subm_pairs) whose
// partial products are atomically added (or, with `partials`, stored per pair).  weight: [Cout, 27, Cin] (spconv [Cout,3,3,3,Cin]).
// pair_off_host: 28 host ints (prefix of pair counts per offset, centre slice empty).
static int subm_conv_impl(int n, int cin, int cout, const float* x, long long ldx, const int* nbr,
                          const float* weight, const float* bias, const int* pair_in, const int* pair_out,
                          const int* pair_off_host, float* out, long long ldo, const unsigned long long* x_amax,
                          unsigned x_tag, const unsigned long long* w_amax, unsigned w_tag, const float* w_split,
                          const float* w_inv, float* partials, long long ldp, void* stream,
                          bool skip_centre = false) {
  SFX_REQUIRE(n >= 0 && cin > 0 && cout > 0, "sfx_subm_conv: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(x && nbr && weight && out && pair_off_host, "sfx_subm_conv: null buffer");
  SFX_REQUIRE(ldx >= cin && ldo >= cout, "sfx_subm_conv: leading dimension too small");
  SFX_REQUIRE(fits(n, ldx) && fits(n, ldo) && fits(cout, 27ll * cin),
              "sfx_subm_conv: operand exceeds the 2 GiB buffer-descriptor range");
  SFX_REQUIRE(!partials || (ldp >= cout && fits(pair_off_host[27], ldp)),
              "sfx_subm_conv_partials: partials leading dimension too small or too large");
  hipStream_t st = sfx::as_stream(stream);
  const bool vec = (cin % 4 == 0) && (ldx % 4 == 0) && aligned16(x) && aligned16(weight);
  // 1) centre offset: dense gathered GEMM with bias, plain stores
  GemmArgs a{};
  a.M = n; a.N = cout; a.K = cin; a.A = x; a.lda = ldx; a.gidx = nbr + 13; a.S = 1; a.Kseg = cin; a.gstride = 27;
  for (const TunedLaunch& t : kTunedConv)  // measured tile shape for both launches of this conv
    if (t.N == cout && t.K == cin && 5ll * n >= 4ll * t.M && 4ll * n <= 5ll * t.M) {
      a.tuned = t.cfg + 1;
      a.tuned_sk = t.sk;
      break;
    }
  a.W = weight + 13ll * cin; a.ldw = 27ll * cin; a.bias = bias; a.act = 0; a.act_ncols = cout; a.Y = out; a.ldy = ldo;
  // fp16x2: one pair of maxima (all of x, all 27 weight slices) for both launches, or the pre-split weight
  a.a_amax = x_amax; a.a_tag = x_tag; a.w_amax = w_amax; a.w_tag = w_tag;
  SFX_REQUIRE(!w_split == !w_inv, "sfx_subm_conv: w_split and w_inv go together");
  if (w_split && vec && aligned16(w_split)) {  // split of the [Cout, 27 * Cin] weight
    a.Wsp = w_split + 13ll * cin; a.ldws = 27ll * cin; a.winv = w_inv;
  }
  if (!a.Wsp && vec && split_mode(cin) == 2 &&
      !prepare_amax(a, AmaxJob{x, ldx, 0, n, cin, 1, nullptr, 0, 1},
                    AmaxJob{weight, 27ll * cin, 0, cout, 27 * cin, 1, nullptr, 0, 1}, st)) {
    a.a_amax = a.w_amax = nullptr;  // (dispatch falls back to bf16x3 for the pair launch)
  }
  if (!skip_centre) {
    dispatch(a, 1, vec, st);
    int rc = sfx::check_launch("sfx_subm_conv(centre)");
    if (rc) return rc;
  }
  if (!pair_in || pair_off_host[27] == 0) return SFX_OK;
  // 2) the other 26 offsets as one flat tile list
  GemmArgs b = a;
  b.gidx = nullptr; b.bias = nullptr; b.gstride = 1; b.pair_mode = 1; b.pair_in = pair_in; b.pair_out = pair_out;
  b.W = weight; b.slice_w_stride = cin; b.num_slices = 27;
  if (a.Wsp) b.Wsp = w_split;
  for (int k = 0; k <= 27; ++k) b.slice_pair_off[k] = pair_off_host[k];
  b.M = pair_off_host[27];
  if (partials) {
    b.pair_store = 1;
    b.Y = partials;
    b.ldy = ldp;
  }
  dispatch(b, 1, vec, st);
  return sfx::check_launch("sfx_subm_conv(pairs)");
}

int sfx_subm_conv(int n, int cin, int cout, const float* x, long long ldx, const int* nbr, const float* weight,
                  const float* bias, const int* pair_in, const int* pair_out, const int* pair_off_host, float* out,
                  long long ldo, const unsigned long long* x_amax, unsigned x_tag,
                  const unsigned long long* w_amax, unsigned w_tag, const float* w_split, const float* w_inv,
                  void* stream) {
  return subm_conv_impl(n, cin, cout, x, ldx, nbr, weight, bias, pair_in, pair_out, pair_off_host, out, ldo, x_amax,
                        x_tag, w_amax, w_tag, w_split, w_inv, nullptr, 0, stream);
}

// Atomic-free form: out = bias + the centre offset's product (plain stores); the 26 other offsets' products are
// stored as rows of `partials` ([num_pairs][ldp], row = pair index in the sfx_subm_pairs lists) for a consumer that
// sums them per output row (sfx_cpe_residual_ln_pairs / sfx_pair_reduce).
int sfx_subm_conv_partials(int n, int cin, int cout, const float* x, long long ldx, const int* nbr,
                           const float* weight, const float* bias, const int* pair_in, const int* pair_out,
                           const int* pair_off_host, float* out, long long ldo, float* partials, long long ldp,
                           const float* w_split, const float* w_inv, void* stream) {
  SFX_REQUIRE(n == 0 || pair_off_host[27] == 0 || (partials && pair_in && pair_out),
              "sfx_subm_conv_partials: null partials / pair lists");
  return subm_conv_impl(n, cin, cout, x, ldx, nbr, weight, bias, pair_in, pair_out, pair_off_host, out, ldo, nullptr,
                        0, nullptr, 0, w_split, w_inv, partials, ldp, stream);
}

// The pair launch of sfx_subm_conv_partials alone (its centre launch made by an earlier sfx_subm_conv_partials call
// with pair_in = NULL): the host can enqueue the centre GEMM before it waits for the pair offsets, so the GPU has
// work while the offsets travel to the host.
int sfx_subm_conv_partials_pairs(int n, int cin, int cout, const float* x, long long ldx, const int* nbr,
                                 const float* weight, const float* bias, const int* pair_in, const int* pair_out,
                                 const int* pair_off_host, float* out, long long ldo, float* partials, long long ldp,
                                 const float* w_split, const float* w_inv, void* stream) {
  SFX_REQUIRE(n == 0 || pair_off_host[27] == 0 || (partials && pair_in && pair_out),
              "sfx_subm_conv_partials_pairs: null partials / pair lists");
  return subm_conv_impl(n, cin, cout, x, ldx, nbr, weight, bias, pair_in, pair_out, pair_off_host, out, ldo, nullptr,
                        0, nullptr, 0, w_split, w_inv, partials, ldp, stream, true);
}

// SubMConv3d backward w.r.t. its input: dX[in] += dY[out] W_k for every pair (in, out, k), centre included.
// weight_t = the [Cout, 27*Cin] weight transposed to [27*Cin, Cout] (sfx_transpose; cached by the caller);
// centre_ws = 2n ints of scratch.  dX is accumulated into (float atomics): zero it or pass the residual
// gradient it should be added to.
int sfx_subm_conv_bwd_data(int n, int cin, int cout, const float* dy, long long ldy, const int* nbr,
                           const float* weight_t, const int* pair_in, const int* pair_out, const int* pair_off_host,
                           int* centre_ws, float* dx, long long lddx, const float* wt_split, const float* wt_inv,
                           void* stream) {
  SFX_REQUIRE(n >= 0 && cin > 0 && cout > 0, "sfx_subm_conv_bwd_data: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(dy && nbr && weight_t && dx && pair_off_host && centre_ws, "sfx_subm_conv_bwd_data: null buffer");
  SFX_REQUIRE(ldy >= cout && lddx >= cin, "sfx_subm_conv_bwd_data: leading dimension too small");
  SFX_REQUIRE(fits(n, ldy) && fits(n, lddx) && fits(27ll * cin, cout),
              "sfx_subm_conv_bwd_data: operand exceeds the 2 GiB buffer-descriptor range");
  hipStream_t st = sfx::as_stream(stream);
  const bool vec = (cout % 4 == 0) && (ldy % 4 == 0) && aligned16(dy) && aligned16(weight_t);
  SFX_REQUIRE(!wt_split == !wt_inv, "sfx_subm_conv_bwd_data: wt_split and wt_inv go together");
  const bool presplit = wt_split && vec && aligned16(wt_split);
  GemmArgs am{};
  if (!presplit && vec && split_mode(cout) == 2)
    (void)prepare_amax(am, AmaxJob{dy, ldy, 0, n, cout, 1, nullptr, 0, 1},
                       AmaxJob{weight_t, (long long)cout, 0, 27 * cin, cout, 1, nullptr, 0, 1}, st);
  int* cg = centre_ws;
  int* cs = centre_ws + n;
  centre_pairs_kernel<<<sfx::ceil_div(n, 256), 256, 0, st>>>(n, nbr, cg, cs);
  GemmArgs a{};
  a.N = cin; a.K = cout; a.A = dy; a.lda = ldy; a.S = 1; a.Kseg = cout; a.gstride = 1;
  a.ldw = cout; a.act = 0; a.act_ncols = cin; a.Y = dx; a.ldy = lddx;
  a.pair_mode = 1; a.slice_w_stride = (long long)cin * cout;
  a.a_amax = am.a_amax; a.a_tag = am.a_tag; a.w_amax = am.w_amax; a.w_tag = am.w_tag;
  if (presplit) { a.ldws = cout; a.winv = wt_inv; a.slice_winv_stride = cin; }
  // centre offset (k = 13) as a one-slice pair launch
  GemmArgs c = a;
  c.pair_in = cg; c.pair_out = cs; c.W = weight_t + 13ll * cin * cout; c.num_slices = 1;
  if (presplit) { c.Wsp = wt_split + 13ll * cin * cout; c.winv = wt_inv + 13ll * cin; }
  c.slice_pair_off[0] = 0; c.slice_pair_off[1] = n; c.M = n;
  dispatch(c, 1, vec, st);
  int rc = sfx::check_launch("sfx_subm_conv_bwd_data(centre)");
  if (rc || !pair_in || pair_off_host[27] == 0) return rc;
  // the 26 other offsets: roles of the forward pair lists swapped
  GemmArgs b = a;
  b.pair_in = pair_out; b.pair_out = pair_in; b.W = weight_t; b.num_slices = 27;
  if (presplit) b.Wsp = wt_split;
  for (int k = 0; k <= 27; ++k) b.slice_pair_off[k] = pair_off_host[k];
  b.M = pair_off_host[27];
  dispatch(b, 1, vec, st);
  return sfx::check_launch("sfx_subm_conv_bwd_data(pairs)");
}

int sfx_linear_bwd_data(int M, int N, int K, const float* dY, long long ldy, const float* Wt, long long ldwt,
                        const float* rowscale, int dact, int dact_ncols, const float* dact_pre, long long ld_pre,
                        float* dX, long long lddx, int accumulate, const float* wt_split, const float* wt_inv,
                        void* stream) {
  SFX_REQUIRE(M >= 0 && N > 0 && K > 0, "sfx_linear_bwd_data: bad sizes M=%d N=%d K=%d", M, N, K);
  SFX_REQUIRE(dact >= 0 && dact <= 3, "sfx_linear_bwd_data: bad dact %d", dact);
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(dY && Wt && dX && (!dact || dact_pre), "sfx_linear_bwd_data: null buffer");
  SFX_REQUIRE(ldy >= N && ldwt >= N && lddx >= K && (!dact || ld_pre >= K), "sfx_linear_bwd_data: leading dim");
  SFX_REQUIRE(fits(M, ldy) && fits(K, ldwt) && fits(M, lddx) && (!dact || fits(M, ld_pre)),
              "sfx_linear_bwd_data: operand exceeds the 2 GiB buffer-descriptor range");
  GemmArgs a{};
  a.M = M; a.N = K; a.K = N; a.A = dY; a.lda = ldy; a.S = 1; a.Kseg = N; a.gstride = 1;
  a.W = Wt; a.ldw = ldwt; a.act = 0; a.act_ncols = dact_ncols < 0 ? K : dact_ncols;
  a.Y = dX; a.ldy = lddx;
  if (accumulate) { a.R = dX; a.ldr = lddx; }
  a.rowscale = rowscale; a.dact = dact; a.dact_pre = dact_pre; a.ld_dact = ld_pre;
  const bool vec = (N % 4 == 0) && (ldy % 4 == 0) && (ldwt % 4 == 0) && aligned16(dY) && aligned16(Wt);
  SFX_REQUIRE(!wt_split == !wt_inv, "sfx_linear_bwd_data: wt_split and wt_inv go together");
  if (wt_split && vec && aligned16(wt_split)) {  // split of Wt [K, N]
    a.Wsp = wt_split; a.ldws = N; a.winv = wt_inv;
  }
  dispatch(a, 1, vec, sfx::as_stream(stream));
  return sfx::check_launch("sfx_linear_bwd_data");
}

int sfx_set_precision(int mode) {
  SFX_REQUIRE(mode == 0 || mode == 1, "sfx_set_precision: mode %d (0 fp32-accurate, 1 reference precision)", mode);
  g_prec = mode;
  return SFX_OK;
}

int sfx_get_precision(void) { return g_prec; }

int sfx_linear_wgrad(int M, int N, int K, const float* dY, long long ldy, const float* X, long long ldx, float* dW,
                     long long ldw, float* db, void* stream) {
  SFX_REQUIRE(M >= 0 && N > 0 && K > 0, "sfx_linear_wgrad: bad sizes M=%d N=%d K=%d", M, N, K);
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(dY && X && dW, "sfx_linear_wgrad: null buffer");
  SFX_REQUIRE(N % 4 == 0 && K % 4 == 0 && ldy % 4 == 0 && ldx % 4 == 0 && aligned16(dY) && aligned16(X),
              "sfx_linear_wgrad: N, K, leading dims must be multiples of 4 and operands 16-byte aligned");
  SFX_REQUIRE(ldy >= N && ldx >= K && ldw >= K, "sfx_linear_wgrad: leading dim");
  SFX_REQUIRE(fits(M, ldy) && fits(M, ldx) && fits(N, ldw), "sfx_linear_wgrad: operand exceeds 2 GiB range");
  hipStream_t st = sfx::as_stream(stream);
  const int slabs = (int)sfx::ceil_div(M, BK);
  if (split_mode(M) != 0) {  // bf16x3 terms, 128 x 128 tiles (SFX_GEMM_PREC=fp32: the exact kernel below)
    const int tiles2 = (int)(sfx::ceil_div(N, WG2_T) * sfx::ceil_div(K, WG2_T));
    int splits2 = (int)sfx::ceil_div(2 * num_cus(), tiles2);
    if (splits2 > slabs) splits2 = slabs;
    if (splits2 < 1) splits2 = 1;
    const int chunk2 = (int)sfx::ceil_div(slabs, splits2) * BK;
    splits2 = (int)sfx::ceil_div(M, chunk2);
    if (g_prec == 1)
      wgrad2_kernel<2><<<dim3(tiles2, splits2), 256, 0, st>>>(M, N, K, dY, ldy, X, ldx, dW, ldw, chunk2, db);
    else
      wgrad2_kernel<3><<<dim3(tiles2, splits2), 256, 0, st>>>(M, N, K, dY, ldy, X, ldx, dW, ldw, chunk2, db);
    return sfx::check_launch("sfx_linear_wgrad");
  }
  const int tiles = (int)(sfx::ceil_div(N, WG_TILE) * sfx::ceil_div(K, WG_TILE));
  int splits = (int)sfx::ceil_div(4 * num_cus(), tiles);
  if (splits > slabs) splits = slabs;
  if (splits < 1) splits = 1;
  const int chunk = (int)sfx::ceil_div(slabs, splits) * BK;
  splits = (int)sfx::ceil_div(M, chunk);
  wgrad_kernel<<<dim3(tiles, splits), THREADS, 0, st>>>(M, N, K, dY, ldy, X, ldx, dW, ldw, chunk, db);
  return sfx::check_launch("sfx_linear_wgrad");
}

int sfx_transpose(int rows, int cols, const float* src, long long lds, float* dst, long long ldd, void* stream) {
  SFX_REQUIRE(rows >= 0 && cols >= 0 && lds >= cols && ldd >= rows, "sfx_transpose: bad sizes");
  if (rows == 0 || cols == 0) return SFX_OK;
  SFX_REQUIRE(src && dst, "sfx_transpose: null buffer");
  transpose_kernel<<<dim3(sfx::ceil_div(cols, 32), sfx::ceil_div(rows, 32)), 256, 0, sfx::as_stream(stream)>>>(
      rows, cols, src, lds, dst, ldd);
  return sfx::check_launch("sfx_transpose");
}

}  // extern "C"
