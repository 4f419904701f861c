// Error plumbing + generic device primitives (scan) shared by every stage.
#include <map>
#include <mutex>
#include <utility>

#include "common.h"

#include <cstring>

namespace sfx {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }

}  // namespace sfx

// ---------------------------------------------------------------------------
// Inclusive / exclusive scans.  int32 (cum_tiles_hit = gsplat's
// torch.cumsum(num_tiles_hit, dtype=int32), every run-length / pair offset in
// the library): one single-pass launch with decoupled look-back (below).
// int64: three launches -- per-block scan (1024 items per 256-thread block), a
// single-workgroup scan of the block totals, then an offset add.
// ---------------------------------------------------------------------------
namespace {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 4;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

template <typename T>
__device__ T block_exclusive_scan(T v, T* smem, T* total) {
  // smem: SCAN_THREADS/64 entries of wave totals
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) smem[wid] = x;
  __syncthreads();
  T wave_off = 0, tot = 0;
  for (int w = 0; w < SCAN_THREADS / 64; ++w) {
    T s = smem[w];
    if (w < wid) wave_off += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wave_off + x - v;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_THREADS) scan_tiles(const T* __restrict__ in, T* __restrict__ out,
                                                           T* __restrict__ tile_sums, long long n, int inclusive) {
  __shared__ T smem[SCAN_THREADS / 64];
  const long long base = (long long)blockIdx.x * SCAN_TILE + (long long)threadIdx.x * SCAN_ITEMS;
  T v[SCAN_ITEMS];
  T s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    v[i] = (base + i < n) ? in[base + i] : (T)0;
    s += v[i];
  }
  T total;
  T excl = block_exclusive_scan<T>(s, smem, &total);
  T run = excl;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    T nv = run + v[i];
    if (base + i < n) out[base + i] = inclusive ? nv : run;
    run = nv;
  }
  if (threadIdx.x == 0 && tile_sums) tile_sums[blockIdx.x] = total;
}

template <typename T>
__global__ void __launch_bounds__(SCAN_THREADS) scan_single(T* __restrict__ data, long long n, T* __restrict__ grand) {
  // exclusive scan of `data` in place, one workgroup, chunked.
  __shared__ T smem[SCAN_THREADS / 64];
  T carry = 0;
  for (long long start = 0; start < n; start += SCAN_TILE) {
    const long long base = start + (long long)threadIdx.x * SCAN_ITEMS;
    T v[SCAN_ITEMS];
    T s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
      v[i] = (base + i < n) ? data[base + i] : (T)0;
      s += v[i];
    }
    T total;
    T excl = block_exclusive_scan<T>(s, smem, &total);
    T run = carry + excl;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
      if (base + i < n) data[base + i] = run;
      run += v[i];
    }
    carry += total;
  }
  if (threadIdx.x == 0 && grand) *grand = carry;
}

template <typename T>
__global__ void add_tile_offsets(T* __restrict__ out, const T* __restrict__ tile_offs, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += tile_offs[i / SCAN_TILE];
}

template <typename T>
int scan_impl(long long n, const T* in, T* out, int inclusive, void* ws, size_t ws_bytes, T* total, hipStream_t st) {
  if (n == 0) {
    if (total) hipMemsetAsync(total, 0, sizeof(T), st);
    return sfx::check_launch("scan");
  }
  const long long tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (ws_bytes < (size_t)tiles * sizeof(T)) {
    sfx::set_error("scan: workspace too small (%zu < %zu)", ws_bytes, (size_t)tiles * sizeof(T));
    return SFX_ERR_WORKSPACE;
  }
  T* sums = reinterpret_cast<T*>(ws);
  scan_tiles<T><<<(unsigned)tiles, SCAN_THREADS, 0, st>>>(in, out, sums, n, inclusive);
  scan_single<T><<<1, SCAN_THREADS, 0, st>>>(sums, tiles, total);
  if (tiles > 1) add_tile_offsets<T><<<sfx::ceil_div(n, 256), 256, 0, st>>>(out, sums, n);
  return sfx::check_launch("scan");
}

// ---- int32: single pass with decoupled look-back --------------------------------------------------------------
// One launch: each 2048-element tile takes a ticket, scans itself, publishes its aggregate, gets its exclusive prefix
// from its predecessors' words (sfx::lb_lookback_wave), publishes its inclusive prefix and writes.  The last tile
// writes the grand total.  The ticket and tile words live in a library-owned area per (device, stream)
// (sfx::lookback_state): the last ticket's holder puts the counter back to 0 and every call tags its words with a
// new epoch, so stale words of earlier scans never match -- no memset per scan.
constexpr int LB_ITEMS = 8;
constexpr int LB_TILE = SCAN_THREADS * LB_ITEMS;
constexpr size_t LB_HEADER = 256;  // ticket counter, then the tile words
constexpr int kLbTimeoutWord = 16;  // header word (u32 index) counting look-back waits that hit the spin cap

__global__ void __launch_bounds__(SCAN_THREADS)
scan_lookback_i32(const int32_t* __restrict__ in, int32_t* __restrict__ out, long long n, int inclusive, int tiles,
                  unsigned* __restrict__ ticket, unsigned long long* __restrict__ flags, int32_t* __restrict__ total,
                  unsigned tag) {
  __shared__ int32_t smem[SCAN_THREADS / 64];
  __shared__ int s_tile, s_prefix;
  if (threadIdx.x == 0) {
    const int t = (int)atomicAdd(ticket, 1u);
    s_tile = t;
    if (t == tiles - 1) atomicExch(ticket, 0u);  // every ticket handed out: ready for the stream's next scan
  }
  __syncthreads();
  const int tile = s_tile;
  const long long base = (long long)tile * LB_TILE + (long long)threadIdx.x * LB_ITEMS;
  int32_t v[LB_ITEMS];
  int32_t s = 0;
  if (base + LB_ITEMS <= n && (((uintptr_t)(in + base)) & 15) == 0) {
    const int4 a = *reinterpret_cast<const int4*>(in + base), b = *reinterpret_cast<const int4*>(in + base + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < LB_ITEMS; ++i) v[i] = (base + i < n) ? in[base + i] : 0;
  }
#pragma unroll
  for (int i = 0; i < LB_ITEMS; ++i) s += v[i];
  int32_t agg;
  const int32_t excl = block_exclusive_scan<int32_t>(s, smem, &agg);
  if (threadIdx.x < 64) {  // wave 0: publish the aggregate, look back, publish the inclusive prefix
    int32_t prefix = 0;
    if (tile == 0) {
      if (threadIdx.x == 0) sfx::lb_store(flags, sfx::lb_word(tag, sfx::kLbPrefix, agg));
    } else {
      if (threadIdx.x == 0) sfx::lb_store(flags + tile, sfx::lb_word(tag, sfx::kLbAgg, agg));
      prefix = sfx::lb_lookback_wave(flags, tile, tag, ticket + kLbTimeoutWord);
      if (threadIdx.x == 0) sfx::lb_store(flags + tile, sfx::lb_word(tag, sfx::kLbPrefix, prefix + agg));
    }
    if (threadIdx.x == 0) {
      s_prefix = prefix;
      if (tile == tiles - 1 && total) *total = prefix + agg;
    }
  }
  __syncthreads();
  int32_t run = s_prefix + excl;
#pragma unroll
  for (int i = 0; i < LB_ITEMS; ++i) {
    const int32_t nv = run + v[i];
    if (base + i < n) out[base + i] = inclusive ? nv : run;
    run = nv;
  }
}

int scan_lookback_impl(long long n, const int32_t* in, int32_t* out, int inclusive, void* ws, size_t ws_bytes,
                       int32_t* total, hipStream_t st) {
  if (n == 0) {
    if (total) hipMemsetAsync(total, 0, sizeof(int32_t), st);
    return sfx::check_launch("scan");
  }
  (void)ws;  // the look-back words live in the stream's library-owned area (sfx::lookback_state)
  (void)ws_bytes;
  const long long tiles = (n + LB_TILE - 1) / LB_TILE;
  unsigned* ticket;
  unsigned long long* flags;
  unsigned tag;
  const int rc = sfx::lookback_state(st, tiles, &ticket, &flags, &tag);
  if (rc != SFX_OK) return rc;
  scan_lookback_i32<<<(unsigned)tiles, SCAN_THREADS, 0, st>>>(in, out, n, inclusive, (int)tiles, ticket, flags,
                                                              total, tag);
  return sfx::check_launch("scan");
}

}  // namespace

namespace sfx {
namespace {
struct LbState {
  unsigned* ticket = nullptr;
  unsigned long long* flags = nullptr;
  long long words = 0;
  unsigned epoch = 0;
};
std::mutex g_lb_mu;
std::map<std::pair<int, hipStream_t>, LbState> g_lb;
constexpr unsigned kLbEpochMax = (1u << 30) - 1;  // lb_tag is 30 bits
}  // namespace

int lookback_state(hipStream_t st, long long words, unsigned** ticket, unsigned long long** flags, unsigned* tag) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return check_launch("look-back state (device)");
  std::lock_guard<std::mutex> lock(g_lb_mu);
  LbState& s = g_lb[{dev, st}];
  if (s.words < words) {  // first use of this stream, or a larger scan: (re)allocate, zeroed in stream order
    const long long w = words > (1ll << 16) ? words : (1ll << 16);
    if (s.ticket) {  // an earlier scan of this stream may still be running on the old area
      if (hipStreamSynchronize(st) != hipSuccess || hipFree(s.ticket) != hipSuccess)
        return check_launch("look-back state (release)");
      s = LbState();
    }
    void* p = nullptr;
    const size_t bytes = 256 + sizeof(unsigned long long) * (size_t)w;
    if (hipMalloc(&p, bytes) != hipSuccess) return check_launch("look-back state (allocate)");
    if (hipMemsetAsync(p, 0, bytes, st) != hipSuccess) return check_launch("look-back state (reset)");
    s.ticket = static_cast<unsigned*>(p);
    s.flags = reinterpret_cast<unsigned long long*>(static_cast<char*>(p) + 256);
    s.words = w;
    s.epoch = 0;
  }
  if (s.epoch == kLbEpochMax) {  // tags about to wrap: clear the words once
    if (hipMemsetAsync(s.flags, 0, sizeof(unsigned long long) * (size_t)s.words, st) != hipSuccess)
      return check_launch("look-back state (epoch wrap)");
    s.epoch = 0;
  }
  *tag = ++s.epoch;
  *ticket = s.ticket;
  *flags = s.flags;
  return SFX_OK;
}

// Look-back waits of this (device, stream)'s area that reached the spin cap since its allocation (0 = every scan
// and radix pass on it was exact); -1: no area (nothing scanned on the stream yet).  Synchronous (host read).
long long lookback_timeouts(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  unsigned* t = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_lb_mu);
    auto it = g_lb.find({dev, st});
    if (it == g_lb.end()) return -1;
    t = it->second.ticket;
  }
  unsigned v = 0;
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipMemcpy(&v, t + kLbTimeoutWord, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return v;
}

// Frees this (device, stream)'s area after the stream's pending work (a caller that destroys a stream it scanned
// on releases its area first; otherwise the area lives as long as the library).
int lookback_release(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return check_launch("look-back release (device)");
  std::lock_guard<std::mutex> lock(g_lb_mu);
  auto it = g_lb.find({dev, st});
  if (it == g_lb.end()) return SFX_OK;
  if (hipStreamSynchronize(st) != hipSuccess || hipFree(it->second.ticket) != hipSuccess)
    return check_launch("look-back release");
  g_lb.erase(it);
  return SFX_OK;
}

// The look-back scan on a given area: `ticket` zero (the kernel puts it back to zero), `flags`
// (lookback_scan_words(n) words) holding no word with this call's `tag` (sfx::lookback_state hands out both).
long long lookback_scan_words(long long n) { return (n + LB_TILE - 1) / LB_TILE; }
void lookback_scan_i32(long long n, const int32_t* in, int32_t* out, int inclusive, unsigned* ticket,
                       unsigned long long* flags, unsigned tag, int32_t* total, hipStream_t st) {
  if (n == 0) return;
  const long long tiles = lookback_scan_words(n);
  scan_lookback_i32<<<(unsigned)tiles, SCAN_THREADS, 0, st>>>(in, out, n, inclusive, (int)tiles, ticket, flags, total,
                                                              tag);
}
}  // namespace sfx

extern "C" {

const char* sfx_last_error(void) { return sfx::g_err; }

int sfx_abi_version(void) { return 16; }

long long sfx_lookback_timeouts(void* stream) { return sfx::lookback_timeouts(sfx::as_stream(stream)); }

int sfx_lookback_release(void* stream) { return sfx::lookback_release(sfx::as_stream(stream)); }

size_t sfx_scan_workspace_bytes(long long n) {
  // int64: one sum per 1024-element tile; int32: the look-back header + one word per 2048-element tile
  const long long tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  const size_t old = (size_t)(tiles > 0 ? tiles : 1) * sizeof(long long);
  const size_t lb = LB_HEADER + (size_t)((n + LB_TILE - 1) / LB_TILE + 1) * sizeof(unsigned long long);
  return old > lb ? old : lb;
}

int sfx_scan_i32(long long n, const int32_t* in, int32_t* out, int inclusive, void* ws, size_t ws_bytes,
                 int32_t* total, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_scan_i32: n < 0");
  SFX_REQUIRE(n == 0 || (in && out), "sfx_scan_i32: null buffer");
  return scan_lookback_impl(n, in, out, inclusive, ws, ws_bytes, total, sfx::as_stream(stream));
}

int sfx_scan_i64(long long n, const int64_t* in, int64_t* out, int inclusive, void* ws, size_t ws_bytes,
                 int64_t* total, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_scan_i64: n < 0");
  SFX_REQUIRE(n == 0 || (in && out), "sfx_scan_i64: null buffer");
  return scan_impl<int64_t>(n, in, out, inclusive, ws, ws_bytes, total, sfx::as_stream(stream));
}

}  // extern "C"
