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
// Per pass: histogram per tile -> exclusive scan over [digit][tile] (one single-pass look-back launch, its
// area reset once per sort and tagged per pass) -> stable rank + LDS reorder + coalesced scatter.  Ranking is wave-local with 8 ballots
// per digit match (wave64 __ballot masks), then a per-wave prefix in LDS.  (A one-sweep form -- per-digit
// look-back inside the scatter, no per-tile histograms -- measured slower here: with every tile resident at once
// the per-digit chains are long; 47.6 vs ~37 us per pass on config B's intersection sort.)
#include "common.h"


namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
constexpr int RS_BINS = 256;

// 8 sub-histograms (lane & 7), padded to 257 words: digits of neighbouring keys are often equal (depth / code high
// bytes), and 64 lanes adding to one LDS word serialise -- with the lanes spread over 8 copies (and the copies over
// banks) the same-address chains are 8x shorter (SQ_LDS_BANK_CONFLICT 88.9 % of LDS cycles with one copy)
constexpr int RS_SUB = 8, RS_SUBW = RS_BINS + 1;
__global__ void __launch_bounds__(RS_THREADS)
radix_hist(const uint64_t* __restrict__ keys, long long n, int shift, int num_tiles, int* __restrict__ hist) {
  __shared__ int h[RS_SUB * RS_SUBW];
  for (int k = threadIdx.x; k < RS_SUB * RS_SUBW; k += RS_THREADS) h[k] = 0;
  __syncthreads();
  const long long base = (long long)blockIdx.x * RS_TILE;
  int* hs = h + (threadIdx.x & (RS_SUB - 1)) * RS_SUBW;
  uint64_t k[RS_ITEMS];
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const long long i = base + (long long)r * RS_THREADS + threadIdx.x;
    k[r] = i < n ? keys[i] : 0ull;
  }
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const long long i = base + (long long)r * RS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&hs[(int)((k[r] >> shift) & 0xff)], 1);
  }
  __syncthreads();
  int c = 0;
#pragma unroll
  for (int q = 0; q < RS_SUB; ++q) c += h[q * RS_SUBW + threadIdx.x];
  hist[(long long)threadIdx.x * num_tiles + blockIdx.x] = c;
}

// Ranking is unchanged (stable: wave-local ballot ranks, waves in order); the pairs are first placed in LDS at their
// tile-local sorted position (digit-major), then written out from LDS in that order, so consecutive lanes store to
// consecutive addresses of each digit's run (runs of ~8 pairs per digit at 2048 pairs per tile) instead of 64
// scattered 8-byte stores per wave instruction.
__global__ void __launch_bounds__(RS_THREADS)
radix_scatter(const uint64_t* __restrict__ keys_in, const int32_t* __restrict__ vals_in, long long n, int shift,
              int num_tiles, const int* __restrict__ offs, uint64_t* __restrict__ keys_out,
              int32_t* __restrict__ vals_out) {
  __shared__ int cnt[RS_WAVES][RS_BINS];
  __shared__ int gdelta[RS_BINS];     // global position - tile-local position, per digit
  __shared__ int wtot[RS_WAVES];
  __shared__ uint64_t sk[RS_TILE];
  __shared__ int32_t sv[RS_TILE];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int k = threadIdx.x; k < RS_WAVES * RS_BINS; k += RS_THREADS) (&cnt[0][0])[k] = 0;
  __syncthreads();

  const long long tbase = (long long)blockIdx.x * RS_TILE;
  const long long wbase = tbase + (long long)wid * 64 * RS_ITEMS;
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
    // digit d = thread: exclusive prefix over the waves (in place), the tile's count of d, then the tile-local run
    // start of d = exclusive scan of the counts over the digits (wave scans + the waves' totals)
    const int d = threadIdx.x;
    int run = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) {
      const int c = cnt[w][d];
      cnt[w][d] = run;
      run += c;
    }
    int incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wtot[wid] = incl;
    __syncthreads();
    int before = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) before += w < wid ? wtot[w] : 0;
    const int lstart = before + incl - run;
    gdelta[d] = offs[(long long)d * num_tiles + blockIdx.x] - lstart;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) cnt[w][d] += lstart;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RS_ITEMS; ++r) {
    const long long i = wbase + (long long)r * 64 + lane;
    if (i < n) {
      const int d = (int)((k_reg[r] >> shift) & 0xff);
      const int lpos = cnt[wid][d] + rank[r];
      sk[lpos] = k_reg[r];
      sv[lpos] = v_reg[r];
    }
  }
  __syncthreads();
  const int tn = (int)min((long long)RS_TILE, n - tbase);
  for (int j = threadIdx.x; j < tn; j += RS_THREADS) {
    const uint64_t k = sk[j];
    const int pos = j + gdelta[(int)((k >> shift) & 0xff)];
    keys_out[pos] = k;
    vals_out[pos] = sv[j];
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
  const long long hist = (tiles > 0 ? tiles : 1) * RS_BINS;
  return align256(sizeof(uint64_t) * (size_t)n) + align256(sizeof(int32_t) * (size_t)n) +
         align256(sizeof(int32_t) * (size_t)hist) + 256 + sizeof(unsigned long long) * (size_t)sfx::lookback_scan_words(hist);
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
  char* p = reinterpret_cast<char*>(ws);
  uint64_t* k_alt = reinterpret_cast<uint64_t*>(p);
  p += align256(sizeof(uint64_t) * (size_t)n);
  int32_t* v_alt = reinterpret_cast<int32_t*>(p);
  p += align256(sizeof(int32_t) * (size_t)n);
  const int tiles = (int)((n + RS_TILE - 1) / RS_TILE);
  const long long hist_n = (long long)tiles * RS_BINS;
  int* hist = reinterpret_cast<int*>(p);
  p += align256(sizeof(int32_t) * (size_t)hist_n);
  // the per-pass digit-count scans run on the stream's library-owned look-back area (no reset per sort)

  const uint64_t* ksrc = keys_in;
  const int32_t* vsrc = vals_in;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = begin_bit + 8 * pass;
    const bool to_out = ((passes - 1 - pass) % 2) == 0;
    uint64_t* kdst = to_out ? keys_out : k_alt;
    int32_t* vdst = to_out ? vals_out : v_alt;
    radix_hist<<<tiles, RS_THREADS, 0, st>>>(ksrc, n, shift, tiles, hist);
    unsigned* ticket;
    unsigned long long* flags;
    unsigned tag;
    const int rc = sfx::lookback_state(st, sfx::lookback_scan_words(hist_n), &ticket, &flags, &tag);
    if (rc != SFX_OK) return rc;
    sfx::lookback_scan_i32(hist_n, hist, hist, 0, ticket, flags, tag, nullptr, st);
    radix_scatter<<<tiles, RS_THREADS, 0, st>>>(ksrc, vsrc, n, shift, tiles, hist, kdst, vdst);
    ksrc = kdst;
    vsrc = vdst;
  }
  return sfx::check_launch("sfx_sort_pairs_u64");
}

}  // extern "C"
