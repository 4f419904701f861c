// Submanifold 3x3x3 neighbour map for the PTv3 CPE (spconv SubMConv3d,
// indice_key=f"stage{s}"; reference models/pointtransformer_v3.py:301-324 ->
// Pointcept Block.cpe).
//
// An open-addressing hash (linear probing, 2^k slots >= 2n) maps the packed
// voxel key (batch, x+1, y+1, z+1) -> lowest point index owning that voxel
// (atomicMin: a deterministic rule for duplicate voxels, where spconv's GPU
// hash picks an arbitrary duplicate).  The query writes nbr[i][k] for the 27
// offsets k = (dx+1)*9 + (dy+1)*3 + (dz+1) (spconv weight layout
// [Cout, kx, ky, kz, Cin], input site = output site + offset), -1 if absent.
// The conv itself is sfx_linear's gathered implicit GEMM over nbr.
#include "common.h"

#include <climits>

namespace {

constexpr unsigned long long EMPTY = ~0ull;

__device__ __forceinline__ unsigned long long pack(int b, int x, int y, int z) {
  return ((unsigned long long)(unsigned)b << 48) | ((unsigned long long)(unsigned)(x + 1) << 32) |
         ((unsigned long long)(unsigned)(y + 1) << 16) | (unsigned long long)(unsigned)(z + 1);
}

__device__ __forceinline__ unsigned slot_of(unsigned long long key, int log2cap) {
  return (unsigned)((key * 0x9E3779B97F4A7C15ull) >> (64 - log2cap));
}

// one launch for the table / mask initialisation (was 2-4 fills): keys EMPTY, vals 0x7f7f7f7f (atomicMin start),
// masks 0
__global__ void subm_init_kernel(long long cap, int n, unsigned long long* __restrict__ keys, int* __restrict__ vals,
                                 unsigned* __restrict__ mask, unsigned long long* __restrict__ mask_keys) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < cap) {
    keys[t] = EMPTY;
    vals[t] = 0x7f7f7f7f;
  }
  if (t < n) {
    if (mask) mask[t] = 0u;
    if (mask_keys) mask_keys[t] = 0ull;
  }
}

__global__ void subm_insert_kernel(int n, const int* __restrict__ grid, const int* __restrict__ batch,
                                   unsigned long long* __restrict__ keys, int* __restrict__ vals, int log2cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long key = pack(batch ? batch[i] : 0, grid[3 * i], grid[3 * i + 1], grid[3 * i + 2]);
  const unsigned mask = (1u << log2cap) - 1u;
  unsigned s = slot_of(key, log2cap);
  while (true) {
    const unsigned long long prev = atomicCAS(&keys[s], EMPTY, key);
    if (prev == EMPTY || prev == key) {
      atomicMin(&vals[s], i);
      return;
    }
    s = (s + 1) & mask;
  }
}

// one thread per (point, offset): 27x the threads of a per-point loop to hide the probe chains' latency, and
// coalesced nbr stores (consecutive threads write consecutive offsets of a point)
__global__ void subm_query_kernel(int n, const int* __restrict__ grid, const int* __restrict__ batch,
                                  const unsigned long long* __restrict__ keys, const int* __restrict__ vals,
                                  int log2cap, int* __restrict__ nbr, unsigned* __restrict__ mask_out,
                                  unsigned long long* __restrict__ mask_keys) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= 27ll * n) return;
  const int i = (int)(q / 27), k = (int)(q - 27ll * i);
  const int x = grid[3 * i] + k / 9 - 1, y = grid[3 * i + 1] + (k / 3) % 3 - 1, z = grid[3 * i + 2] + k % 3 - 1;
  const unsigned cmask = (1u << log2cap) - 1u;
  int out = -1;
  if (x >= 0 && y >= 0 && z >= 0) {
    const unsigned long long key = pack(batch ? batch[i] : 0, x, y, z);
    unsigned s = slot_of(key, log2cap);
    while (true) {
      const unsigned long long kk = keys[s];
      if (kk == key) {
        out = vals[s];
        break;
      }
      if (kk == EMPTY) break;
      s = (s + 1) & cmask;
    }
  }
  nbr[q] = out;
  if (out >= 0) {  // (masks zeroed by the launcher)
    if (mask_out) atomicOr(&mask_out[i], 1u << k);
    if (mask_keys) atomicOr(&mask_keys[i], 1ull << k);
  }
}

// rows of nbr / mask in mask-sorted order (perm from a radix sort of the masks)
__global__ void subm_permute_kernel(int n, const int* __restrict__ perm, const int* __restrict__ nbr,
                                    const unsigned* __restrict__ mask, int* __restrict__ nbr_sorted,
                                    unsigned* __restrict__ mask_sorted) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 27ll * n) return;
  const int p = (int)(t / 27), k = (int)(t - 27ll * p);
  const int src = perm[p];
  nbr_sorted[t] = nbr[27ll * src + k];
  if (k == 0) mask_sorted[p] = mask[src];
}

// offset-major pair lists (spconv indice pairs, centre offset excluded): flags over [27][n]
// (with_centre: the centre offset k = 13 is listed too -- the eval conv's single pair launch)
__global__ void subm_pair_flags_kernel(int n, const int* __restrict__ nbr, int* __restrict__ flags, int with_centre) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 27ll * n) return;
  const int k = (int)(t / n), i = (int)(t - (long long)k * n);
  flags[t] = ((k != 13 || with_centre) && nbr[27ll * i + k] >= 0) ? 1 : 0;
}

__global__ void subm_pair_fill_kernel(int n, const int* __restrict__ nbr, const int* __restrict__ flags,
                                      const int* __restrict__ pos, int* __restrict__ pair_in,
                                      int* __restrict__ pair_out, int* __restrict__ pair_off) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 27ll * n) return;
  const int k = (int)(t / n), i = (int)(t - (long long)k * n);
  if (i == 0) pair_off[k] = pos[t];
  if (flags[t]) {
    const int p = pos[t];
    pair_out[p] = i;
    pair_in[p] = nbr[27ll * i + k];
  }
}

// inverted pair index: pair_pos[out][k] = index of pair (k, out) in the flat lists (-1: none; centre -1)
__global__ void subm_pair_pos_kernel(long long num_pairs, const int* __restrict__ pair_out,
                                     const int* __restrict__ pair_off, int* __restrict__ pair_pos) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= num_pairs) return;
  int k = 0;
#pragma unroll 1
  for (int q = 1; q < 27; ++q)
    if (pair_off[q] <= p) k = q;
  pair_pos[27ll * pair_out[p] + k] = (int)p;
}

// ---- pair lists by block counts (sfx_subm_pair_lists) ----------------------------------------------------------
// Workgroup b owns points [256 b, 256 b + 256) and reads each point's 27 neighbours once (row-major, the layout nbr is
// written in).  Pass 1 counts the pairs of every (offset k, workgroup b); one scan over those 27 x nb counts gives
// each (k, b) its first slot; pass 2 writes the pairs at that slot + the wave's offset + the lane's rank (ballot +
// mbcnt), so within an offset the pairs stay in ascending output order, and writes the inverted index pair_pos
// [n][27] on the way.  (The flag / scan / fill form scanned 27 n flags and read nbr transposed.)
__device__ __forceinline__ bool pair_flag(const int* row, int k, bool in, int with_centre) {
  return in && (k != 13 || with_centre) && row[k] >= 0;
}
__global__ void __launch_bounds__(256) subm_pair_count_kernel(int n, const int* __restrict__ nbr,
                                                              int* __restrict__ counts, int nb, int with_centre) {
  __shared__ int wc[27][4];
  const int i = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool in = i < n;
  const int* row = nbr + 27ll * (in ? i : 0);
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    const unsigned long long bal = __ballot(pair_flag(row, k, in, with_centre));
    if (lane == 0) wc[k][wid] = __popcll(bal);
  }
  __syncthreads();
  if (threadIdx.x < 27) {
    const int k = threadIdx.x;
    counts[(long long)k * nb + blockIdx.x] = wc[k][0] + wc[k][1] + wc[k][2] + wc[k][3];
  }
}
__global__ void __launch_bounds__(256) subm_pair_write_kernel(int n, const int* __restrict__ nbr,
                                                              const int* __restrict__ first, int nb, int with_centre,
                                                              int* __restrict__ pair_in, int* __restrict__ pair_out,
                                                              int* __restrict__ pair_off, int* __restrict__ pair_pos,
                                                              int* __restrict__ pair_cpos) {
  __shared__ int wc[27][4];
  const int i = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool in = i < n;
  const int* row = nbr + 27ll * (in ? i : 0);
  unsigned long long bal[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    bal[k] = __ballot(pair_flag(row, k, in, with_centre));
    if (lane == 0) wc[k][wid] = __popcll(bal[k]);
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 27) pair_off[threadIdx.x] = first[(long long)threadIdx.x * nb];
  int pk[27], rank[27], cnt = 0;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    int base = first[(long long)k * nb + blockIdx.x];
    for (int w = 0; w < wid; ++w) base += wc[k][w];
    const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(bal[k] >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)bal[k], 0u));
    const bool fl = (bal[k] >> lane) & 1ull;
    const int p = base + (int)rank;
    if (fl) {
      pair_out[p] = i;
      pair_in[p] = row[k];
    }
    if (pair_pos && in) pair_pos[27ll * i + k] = fl ? p : -1;
    pk[k] = fl ? p : -1;
    rank[k] = cnt;
    cnt += fl ? 1 : 0;
  }
  if (pair_cpos && in) {  // compacted: the present pairs in ascending offset order (selects, no register indexing)
    int c[32];
#pragma unroll
    for (int q = 0; q < 31; ++q) c[q] = -1;
#pragma unroll
    for (int k = 0; k < 27; ++k)
#pragma unroll
      for (int q = 0; q <= k; ++q) c[q] = (pk[k] >= 0 && rank[k] == q) ? pk[k] : c[q];
    c[31] = cnt;
    int4* dst = reinterpret_cast<int4*>(pair_cpos + 32ll * i);
#pragma unroll
    for (int q = 0; q < 8; ++q) dst[q] = make_int4(c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]);
  }
}
}  // namespace

extern "C" int sfx_scan_i32(long long n, const int32_t* in, int32_t* out, int inclusive, void* ws, size_t ws_bytes,
                            int32_t* total, void* stream);
extern "C" size_t sfx_scan_workspace_bytes(long long n);

extern "C" {

int sfx_subm_table_log2(int n) {
  int l = 4;
  while ((1ll << l) < 2ll * (n > 0 ? n : 1)) ++l;
  return l;
}

// table_keys: 2^log2cap u64, table_vals: 2^log2cap i32 (both scratch); nbr: [n][27] i32
int sfx_subm_neighbors(int n, const int* grid_coord, const int* batch, int log2cap, unsigned long long* table_keys,
                       int* table_vals, int* nbr, unsigned* mask, unsigned long long* mask_keys, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_subm_neighbors: n < 0");
  SFX_REQUIRE(log2cap >= 4 && log2cap <= 31 && (1ll << log2cap) >= 2ll * n, "sfx_subm_neighbors: table too small");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(grid_coord && table_keys && table_vals && nbr, "sfx_subm_neighbors: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  const size_t cap = (size_t)1 << log2cap;
  subm_init_kernel<<<sfx::ceil_div((long long)cap, 256), 256, 0, st>>>((long long)cap, n, table_keys, table_vals, mask,
                                                                       mask_keys);  // (cap >= 2n)
  subm_insert_kernel<<<sfx::ceil_div(n, 256), 256, 0, st>>>(n, grid_coord, batch, table_keys, table_vals, log2cap);
  subm_query_kernel<<<sfx::ceil_div(27ll * n, 256), 256, 0, st>>>(n, grid_coord, batch, table_keys, table_vals,
                                                                  log2cap, nbr, mask, mask_keys);
  return sfx::check_launch("sfx_subm_neighbors");
}

// pair lists for sfx_subm_conv: pair_in/pair_out hold up to 26*n entries (27*n with_centre); pair_off[28] (device)
// receives the per-offset prefix (centre slice empty unless with_centre).  ws: 2 * 27 * n int32 + sfx_scan_workspace_bytes(27 * n).
size_t sfx_subm_pairs_workspace_bytes(int n) {
  const long long e = 27ll * (n > 0 ? n : 1);
  return (size_t)(2 * e * sizeof(int) + 256) + sfx_scan_workspace_bytes(e);
}

int sfx_subm_pairs(int n, const int* nbr, void* ws, size_t ws_bytes, int* pair_in, int* pair_out, int* pair_off,
                   int with_centre, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_subm_pairs: n < 0");
  SFX_REQUIRE(ws_bytes >= sfx_subm_pairs_workspace_bytes(n), "sfx_subm_pairs: workspace too small");
  SFX_REQUIRE(pair_off, "sfx_subm_pairs: null pair_off");
  hipStream_t st = sfx::as_stream(stream);
  if (n == 0) {
    hipMemsetAsync(pair_off, 0, 28 * sizeof(int), st);
    return sfx::check_launch("sfx_subm_pairs");
  }
  SFX_REQUIRE(nbr && ws && pair_in && pair_out, "sfx_subm_pairs: null buffer");
  const long long e = 27ll * n;
  int* flags = reinterpret_cast<int*>(ws);
  int* pos = flags + e;
  char* scan_ws = reinterpret_cast<char*>(pos + e);
  scan_ws += (256 - (reinterpret_cast<uintptr_t>(scan_ws) & 255)) & 255;
  subm_pair_flags_kernel<<<sfx::ceil_div(e, 256), 256, 0, st>>>(n, nbr, flags, with_centre);
  int rc = sfx_scan_i32(e, flags, pos, 0, scan_ws, sfx_scan_workspace_bytes(e), pair_off + 27, stream);
  if (rc) return rc;
  subm_pair_fill_kernel<<<sfx::ceil_div(e, 256), 256, 0, st>>>(n, nbr, flags, pos, pair_in, pair_out, pair_off);
  return sfx::check_launch("sfx_subm_pairs");
}

// sfx_subm_pairs' lists (same order, same pair_off) plus, when pair_pos is not null, the inverted index pair_pos [n][27]
// of sfx_subm_pair_pos -- by per-workgroup counts (two passes over nbr, a scan of 27 * ceil(n / 256) counts)
size_t sfx_subm_pair_lists_workspace_bytes(int n) {
  const long long e = 27ll * sfx::ceil_div(n > 0 ? n : 1, 256);
  return (size_t)(2 * e * sizeof(int) + 256) + sfx_scan_workspace_bytes(e);
}
int sfx_subm_pair_lists(int n, const int* nbr, void* ws, size_t ws_bytes, int* pair_in, int* pair_out, int* pair_off,
                        int* pair_pos, int* pair_cpos, int with_centre, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_subm_pair_lists: n < 0");
  SFX_REQUIRE(ws_bytes >= sfx_subm_pair_lists_workspace_bytes(n), "sfx_subm_pair_lists: workspace too small");
  SFX_REQUIRE(pair_off, "sfx_subm_pair_lists: null pair_off");
  hipStream_t st = sfx::as_stream(stream);
  if (n == 0) {
    hipMemsetAsync(pair_off, 0, 28 * sizeof(int), st);
    return sfx::check_launch("sfx_subm_pair_lists");
  }
  SFX_REQUIRE(nbr && ws && pair_in && pair_out, "sfx_subm_pair_lists: null buffer");
  const int nb = (int)sfx::ceil_div(n, 256);
  const long long e = 27ll * nb;
  int* counts = reinterpret_cast<int*>(ws);
  int* first = counts + e;
  char* scan_ws = reinterpret_cast<char*>(first + e);
  scan_ws += (256 - (reinterpret_cast<uintptr_t>(scan_ws) & 255)) & 255;
  subm_pair_count_kernel<<<nb, 256, 0, st>>>(n, nbr, counts, nb, with_centre);
  const int rc = sfx_scan_i32(e, counts, first, 0, scan_ws, sfx_scan_workspace_bytes(e), pair_off + 27, stream);
  if (rc) return rc;
  subm_pair_write_kernel<<<nb, 256, 0, st>>>(n, nbr, first, nb, with_centre, pair_in, pair_out, pair_off, pair_pos,
                                             pair_cpos);
  return sfx::check_launch("sfx_subm_pair_lists");
}
// pair_pos [n][27]: for output row i and offset k, the index of pair (k, i) in pair_in/pair_out (-1: no pair);
// pair_off (device, 28 ints) as written by sfx_subm_pairs, num_pairs = pair_off[27]
int sfx_subm_pair_pos(int n, long long num_pairs, const int* pair_out, const int* pair_off, int* pair_pos,
                      void* stream) {
  SFX_REQUIRE(n >= 0 && num_pairs >= 0 && num_pairs <= 26ll * n, "sfx_subm_pair_pos: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(pair_pos && (num_pairs == 0 || (pair_out && pair_off)), "sfx_subm_pair_pos: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  hipMemsetAsync(pair_pos, 0xff, 27ll * n * sizeof(int), st);
  if (num_pairs > 0)
    subm_pair_pos_kernel<<<sfx::ceil_div(num_pairs, 256), 256, 0, st>>>(num_pairs, pair_out, pair_off, pair_pos);
  return sfx::check_launch("sfx_subm_pair_pos");
}

int sfx_subm_permute(int n, const int* perm, const int* nbr, const unsigned* mask, int* nbr_sorted,
                     unsigned* mask_sorted, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_subm_permute: n < 0");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(perm && nbr && mask && nbr_sorted && mask_sorted, "sfx_subm_permute: null buffer");
  subm_permute_kernel<<<sfx::ceil_div(27ll * n, 256), 256, 0, sfx::as_stream(stream)>>>(n, perm, nbr, mask,
                                                                                        nbr_sorted, mask_sorted);
  return sfx::check_launch("sfx_subm_permute");
}

}  // extern "C"
