// Stable LSD radix sort of (u64 key, i32 value) pairs, 8-bit digits.
//
// Replaces the torch.sort / torch.argsort calls on the hot path:
//   * gsplat bin_and_sort_gaussians: torch.sort(isect_ids) (reference
//     utils/gs_utils.py:96 -> gsplat v0.1.11, a stable CUB radix sort on CUDA),
//   * Pointcept Point.serialization / SerializedPooling: torch.argsort(code)
//     and torch.sort(cluster) (reference models/pointtransformer_v3.py:380,
//     :290-299).
// Stability matters: equal keys keep input order, which is what the CUDA
// radix sorts the reference relies on produce.
//
// One sweep per 8-bit digit (Adinets & Merrill's onesweep, re-derived for wave64): a single histogram launch
// reads the keys once and counts every pass's digits (global [pass][256] counts); then each pass is ONE launch:
// a 2048-key tile takes a ticket, ranks its keys per wave (8 ballots per digit match, per-wave prefix in LDS),
// publishes its per-digit counts, gets every digit's exclusive prefix over the preceding tiles by decoupled
// look-back (one thread per digit, sfx::lb_lookback_thread), publishes its inclusive prefixes and scatters.
// The workspace's look-back words are tagged with the pass, so one memset per sort resets all of them.
#include "common.h"

#include <algorithm>


namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
constexpr int RS_BINS = 256;

constexpr int RS_MAX_PASSES = 8;
// workspace: [tickets[8] u32 | pad] [hist[8][256] i32] [flags[tiles][256] u64]
constexpr size_t RS_HDR = 64;
constexpr size_t RS_HIST = RS_MAX_PASSES * RS_BINS * sizeof(int);

// every pass's digit histogram in one read of the keys (per-workgroup LDS counts, then one atomic per bin)
__global__ void __launch_bounds__(RS_THREADS)
radix_hist_all(const uint64_t* __restrict__ keys, long long n, int begin_bit, int passes, int* __restrict__ hist) {
  __shared__ int h[RS_MAX_PASSES][RS_BINS];
  for (int k = threadIdx.x; k < RS_MAX_PASSES * RS_BINS; k += RS_THREADS) (&h[0][0])[k] = 0;
  __syncthreads();
  const long long stride = (long long)gridDim.x * RS_THREADS;
  for (long long i = (long long)blockIdx.x * RS_THREADS + threadIdx.x; i < n; i += stride) {
    const uint64_t k = keys[i] >> begin_bit;
    for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(int)((k >> (8 * p)) & 0xff)], 1);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < passes * RS_BINS; k += RS_THREADS) {
    const int c = (&h[0][0])[k];
    if (c) atomicAdd(hist + k, c);
  }
}

__global__ void __launch_bounds__(RS_THREADS)
radix_onesweep(const uint64_t* __restrict__ keys_in, const int32_t* __restrict__ vals_in, long long n, int shift,
               int pass, unsigned* __restrict__ tickets, const int* __restrict__ hist,
               unsigned long long* __restrict__ flags, uint64_t* __restrict__ keys_out, int32_t* __restrict__ vals_out) {
  __shared__ int cnt[RS_WAVES][RS_BINS];
  __shared__ int base[RS_BINS];
  __shared__ int wsum[RS_WAVES];
  __shared__ int s_tile;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_tile = (int)atomicAdd(tickets + pass, 1u);
  for (int k = threadIdx.x; k < RS_WAVES * RS_BINS; k += RS_THREADS) (&cnt[0][0])[k] = 0;
  {
    // global exclusive digit offsets of this pass (the histogram launch finished before this one)
    const int c = hist[pass * RS_BINS + threadIdx.x];
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int off = 0;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    base[threadIdx.x] = off + x - c;
  }
  __syncthreads();
  const int tile = s_tile;

  const long long wbase = (long long)tile * RS_TILE + (long long)wid * 64 * RS_ITEMS;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint64_t k_reg[RS_ITEMS];
  int32_t v_reg[RS_ITEMS];
  int rank[RS_ITEMS];
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const long long i = wbase + (long long)r * 64 + lane;
    const bool valid = i < n;
    uint64_t k = valid ? keys_in[i] : 0ull;
    k_reg[r] = k;
    v_reg[r] = valid ? (vals_in ? vals_in[i] : (int32_t)i) : 0;
    const int d = (int)((k >> shift) & 0xff);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const unsigned long long bal = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bal : ~bal;
    }
    const int pre = cnt[wid][d];
    const int leader = __ffsll((long long)peers) - 1;
    rank[r] = pre + __popcll(peers & lt_mask);
    if (valid && lane == leader) cnt[wid][d] = pre + __popcll(peers);
  }
  __syncthreads();
  {
    // digit d: this tile's count -> publish, look back, publish the inclusive prefix; then per-wave offsets
    const int d = threadIdx.x;
    int agg = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) agg += cnt[w][d];
    const unsigned tag = (unsigned)pass + 1u;
    unsigned long long* my = flags + (long long)tile * RS_BINS + d;
    int excl = 0;
    if (tile == 0) {
      sfx::lb_store(my, sfx::lb_word(tag, sfx::kLbPrefix, agg));
    } else {
      sfx::lb_store(my, sfx::lb_word(tag, sfx::kLbAgg, agg));
      excl = sfx::lb_lookback_thread(flags + d, RS_BINS, tile, tag);
      sfx::lb_store(my, sfx::lb_word(tag, sfx::kLbPrefix, excl + agg));
    }
    int run = base[d] + excl;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) {
      const int c = cnt[w][d];
      cnt[w][d] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const long long i = wbase + (long long)r * 64 + lane;
    if (i < n) {
      const int d = (int)((k_reg[r] >> shift) & 0xff);
      const int pos = cnt[wid][d] + rank[r];
      keys_out[pos] = k_reg[r];
      vals_out[pos] = v_reg[r];
    }
  }
}

__global__ void iota_copy(const uint64_t* __restrict__ kin, const int32_t* __restrict__ vin, long long n,
                          uint64_t* __restrict__ kout, int32_t* __restrict__ vout) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    kout[i] = kin[i];
    vout[i] = vin ? vin[i] : (int32_t)i;
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

size_t sfx_sort_workspace_bytes(long long n) {
  const long long tiles = (n + RS_TILE - 1) / RS_TILE;
  return align256(sizeof(uint64_t) * (size_t)n) + align256(sizeof(int32_t) * (size_t)n) + RS_HDR + RS_HIST +
         sizeof(unsigned long long) * (size_t)(tiles > 0 ? tiles : 1) * RS_BINS;
}

// Sort `n` pairs by bits [begin_bit, end_bit) of the key (stable).  vals_in may
// be NULL: values are then the input positions (argsort).  keys_in/vals_in are
// not modified.  keys_out/vals_out must not alias the inputs.
int sfx_sort_pairs_u64(long long n, const uint64_t* keys_in, const int32_t* vals_in, uint64_t* keys_out,
                       int32_t* vals_out, int begin_bit, int end_bit, void* ws, size_t ws_bytes, void* stream) {
  SFX_REQUIRE(n >= 0 && n < (1ll << 31), "sfx_sort_pairs_u64: n out of range");
  SFX_REQUIRE(begin_bit >= 0 && end_bit <= 64 && begin_bit <= end_bit, "sfx_sort_pairs_u64: bad bit range");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(keys_in && keys_out && vals_out, "sfx_sort_pairs_u64: null buffer");
  SFX_REQUIRE(ws_bytes >= sfx_sort_workspace_bytes(n), "sfx_sort_pairs_u64: workspace too small");
  hipStream_t st = sfx::as_stream(stream);
  const int passes = (end_bit - begin_bit + 7) / 8;
  if (passes == 0) {
    iota_copy<<<sfx::ceil_div(n, 256), 256, 0, st>>>(keys_in, vals_in, n, keys_out, vals_out);
    return sfx::check_launch("sfx_sort_pairs_u64");
  }
  SFX_REQUIRE(passes <= RS_MAX_PASSES, "sfx_sort_pairs_u64: too many digit passes");
  char* p = reinterpret_cast<char*>(ws);
  uint64_t* k_alt = reinterpret_cast<uint64_t*>(p);
  p += align256(sizeof(uint64_t) * (size_t)n);
  int32_t* v_alt = reinterpret_cast<int32_t*>(p);
  p += align256(sizeof(int32_t) * (size_t)n);
  const int tiles = (int)((n + RS_TILE - 1) / RS_TILE);
  unsigned* tickets = reinterpret_cast<unsigned*>(p);
  int* hist = reinterpret_cast<int*>(p + RS_HDR);
  unsigned long long* flags = reinterpret_cast<unsigned long long*>(p + RS_HDR + RS_HIST);
  // one reset per sort: tickets, histograms and the look-back words (tagged per pass)
  if (hipMemsetAsync(p, 0, RS_HDR + RS_HIST + sizeof(unsigned long long) * (size_t)tiles * RS_BINS, st) != hipSuccess)
    return sfx::check_launch("sfx_sort_pairs_u64 (workspace reset)");
  const int hist_blocks = (int)std::min<long long>(tiles, 1024);
  radix_hist_all<<<hist_blocks, RS_THREADS, 0, st>>>(keys_in, n, begin_bit, passes, hist);
  const uint64_t* ksrc = keys_in;
  const int32_t* vsrc = vals_in;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = begin_bit + 8 * pass;
    const bool to_out = ((passes - 1 - pass) % 2) == 0;
    uint64_t* kdst = to_out ? keys_out : k_alt;
    int32_t* vdst = to_out ? vals_out : v_alt;
    radix_onesweep<<<tiles, RS_THREADS, 0, st>>>(ksrc, vsrc, n, shift, pass, tickets, hist, flags, kdst, vdst);
    ksrc = kdst;
    vsrc = vdst;
  }
  return sfx::check_launch("sfx_sort_pairs_u64");
}

}  // extern "C"
