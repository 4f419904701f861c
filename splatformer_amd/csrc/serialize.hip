// Point serialization and serialized pooling (Pointcept PTv3 m1 semantics,
// reference models/pointtransformer_v3.py:130 orders ("z","z-trans",
// "hilbert","hilbert-trans"), :380 Point.serialization, :290-299
// SerializedPooling).
//
// Codes are computed per point in registers (bit interleave for z-order, the
// Skilling transform as integer bit ops for Hilbert), all orders are sorted
// in ONE stable radix sort by prefixing the order index above the code bits,
// and a finalize pass writes order/inverse.  Pooling sorts code[0] by its
// bits above 3*pooling_depth (== torch.unique + sort(cluster)), marks run
// heads, scans them into cluster ids and reduces features per run.
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace {

// ---- z-order (OCNN KeyLUT xyz2key): bit i of x -> 3i+2, y -> 3i+1, z -> 3i
__device__ __forceinline__ uint64_t z_encode(uint32_t x, uint32_t y, uint32_t z, int depth) {
  uint64_t key = 0;
  for (int i = 0; i < depth; ++i) {
    key |= (uint64_t)((x >> i) & 1u) << (3 * i + 2);
    key |= (uint64_t)((y >> i) & 1u) << (3 * i + 1);
    key |= (uint64_t)((z >> i) & 1u) << (3 * i + 0);
  }
  return key;
}

// ---- Hilbert (Pointcept hilbert.encode, Skilling 2004), locs = (x,y,z) -> dims 0,1,2
__device__ __forceinline__ uint64_t hilbert_encode(uint32_t x, uint32_t y, uint32_t z, int nb) {
  uint32_t g[3] = {x & ((1u << nb) - 1u), y & ((1u << nb) - 1u), z & ((1u << nb) - 1u)};
  for (int bit = 0; bit < nb; ++bit) {
    const int pos = nb - 1 - bit;          // bit index (MSB-first position `bit`)
    const uint32_t low = (1u << pos) - 1u;  // positions bit+1 .. nb-1 (lower bits)
    for (int d = 0; d < 3; ++d) {
      const uint32_t m = (g[d] >> pos) & 1u;
      if (m) {
        g[0] ^= low;
      } else {
        const uint32_t t = (g[0] ^ g[d]) & low;
        g[d] ^= t;
        g[0] ^= t;
      }
    }
  }
  // interleave MSB-first as [bit][dim] (dim 0 most significant in a triplet)
  uint64_t gray = 0;
  for (int k = 0; k < nb; ++k) {
    const int pos = nb - 1 - k;
    for (int d = 0; d < 3; ++d) gray = (gray << 1) | ((g[d] >> pos) & 1u);
  }
  // gray -> binary: prefix xor from the MSB
  uint64_t b = gray;
  b ^= b >> 1;
  b ^= b >> 2;
  b ^= b >> 4;
  b ^= b >> 8;
  b ^= b >> 16;
  b ^= b >> 32;
  return b;
}

__device__ __forceinline__ uint64_t encode_order(int type, int x, int y, int z, int depth) {
  switch (type) {
    case 0: return z_encode(x, y, z, depth);
    case 1: return z_encode(y, x, z, depth);
    case 2: return hilbert_encode(x, y, z, depth);
    default: return hilbert_encode(y, x, z, depth);
  }
}

__global__ void serialize_keys_kernel(int n, const int* __restrict__ grid, const int* __restrict__ batch, int depth,
                                      int num_orders, int4 types, int code_bits, int64_t* __restrict__ codes,
                                      uint64_t* __restrict__ keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int x = grid[3 * i], y = grid[3 * i + 1], z = grid[3 * i + 2];
  const uint64_t b = batch ? (uint64_t)batch[i] : 0ull;
  const int t[4] = {types.x, types.y, types.z, types.w};
  for (int r = 0; r < num_orders; ++r) {
    const uint64_t code = (b << (3 * depth)) | encode_order(t[r], x, y, z, depth);
    codes[(long long)r * n + i] = (int64_t)code;
    keys[(long long)r * n + i] = ((uint64_t)r << code_bits) | code;
  }
}

// sorted positions of the R*n combined keys -> order[r][p], inverse[r][i]
__global__ void serialize_finalize_kernel(int n, int R, const int* __restrict__ sorted_pos, int* __restrict__ order,
                                          int* __restrict__ inverse) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long long)R * n) return;
  const int r = (int)(q / n), p = (int)(q - (long long)r * n);
  const int i = sorted_pos[q] - r * n;
  order[q] = i;
  inverse[(long long)r * n + i] = p;
}

// ---- pooling -------------------------------------------------------------
// Sort-free SerializedPooling.  Every order type's code is hierarchical: code_r(g) >> 3pd == code_r(g >> pd) at
// depth - pd (z-order and Hilbert alike, batch bits on top), so along the parent's sorted order of row r the
// points of one coarse cell (= one cluster) are contiguous and the runs appear in ascending pooled-code order.
// Run starts therefore give torch.unique(code[0] >> 3pd) (row0) and the argsort of the pooled codes (every row)
// without sorting anything.  Each row holds exactly m runs; the host checks that before the assign kernels run.
__global__ void pool_run_flags_kernel(int n, int R, const int* __restrict__ order, const int64_t* __restrict__ codes,
                                      int shift, int* __restrict__ flags) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long long)R * n) return;
  const int r = (int)(q / n), j = (int)(q - (long long)r * n);
  const int64_t* cr = codes + (long long)r * n;
  const uint64_t c = (uint64_t)cr[order[q]] >> shift;
  flags[q] = (j == 0 || c != ((uint64_t)cr[order[q - 1]] >> shift)) ? 1 : 0;
}

// Run counts of code >> shift_k along one serialized row for up to 8 shifts at once (every pooling's cluster count
// from the stage-0 codes, PointTransformerV3.forward): counts[k] += the flags of pool_run_flags_kernel, summed per
// wave by ballot + popcount and per workgroup in LDS, one integer atomic per (workgroup, shift) -- one launch
// instead of a flag pass + scan per pooling (the count is a sum, not a prefix).
struct RunShifts {
  int s[8];
};
__global__ void __launch_bounds__(256) pool_run_counts_kernel(int n, const int* __restrict__ order,
                                                              const int64_t* __restrict__ codes, RunShifts sh,
                                                              int nshift, int* __restrict__ counts) {
  __shared__ int part[8];
  if (threadIdx.x < 8) part[threadIdx.x] = 0;
  __syncthreads();
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t c = 0, p = 0;
  if (j < n) {
    c = (uint64_t)codes[order[j]];
    if (j > 0) p = (uint64_t)codes[order[j - 1]];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k >= nshift) break;
    const bool f = j < n && (j == 0 || (c >> sh.s[k]) != (p >> sh.s[k]));
    const int cnt = __popcll(__ballot(f));
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&part[k], cnt);
  }
  __syncthreads();
  if (threadIdx.x < nshift && part[threadIdx.x]) atomicAdd(counts + threadIdx.x, part[threadIdx.x]);
}

// row0's runs -> cluster id of every point, CSR of the members (sidx / idx_ptr), one head per cluster
__global__ void pool_assign_runs_kernel(int n, int m, int row0, const int* __restrict__ order,
                                        const int* __restrict__ pos, const int* __restrict__ flags,
                                        int* __restrict__ cluster, int* __restrict__ idx_ptr, int* __restrict__ head,
                                        int* __restrict__ sidx) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const long long q = (long long)row0 * n + j;
  const int p = order[q];
  const int c = pos[q] - 1 - row0 * m;
  cluster[p] = c;
  sidx[j] = p;
  // a run index past m (codes that are not hierarchical: the caller's deferred run check raises) is never used
  // as an address
  if (flags[q] && (unsigned)c < (unsigned)m) {
    idx_ptr[c] = j;
    head[c] = p;
  }
  if (j == n - 1) idx_ptr[m] = n;
}

// every row's runs -> order / inverse of the pooled points (the argsort of the pooled codes)
__global__ void pool_reorder_kernel(int n, int m, int R, const int* __restrict__ order, const int* __restrict__ pos,
                                    const int* __restrict__ flags, const int* __restrict__ cluster,
                                    int* __restrict__ new_order, int* __restrict__ new_inverse) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long long)R * n || !flags[q]) return;
  const int r = (int)(q / n);
  const int k = pos[q] - 1 - r * m;
  const int c = cluster[order[q]];
  if ((unsigned)k >= (unsigned)m || (unsigned)c >= (unsigned)m) return;  // (see pool_assign_runs_kernel)
  new_order[(long long)r * m + k] = c;
  new_inverse[(long long)r * m + c] = k;
}

// new codes / grid / batch of the pooled point; keys for the combined sort
__global__ void pool_gather_kernel(int m, int n, int R, const int* __restrict__ head, const int64_t* __restrict__ codes,
                                   int pd, const int* __restrict__ grid, const int* __restrict__ batch,
                                   const float* __restrict__ coord, int code_bits, int64_t* __restrict__ new_codes,
                                   uint64_t* __restrict__ keys, int* __restrict__ new_grid,
                                   int* __restrict__ new_batch) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= m) return;
  const int hd = head[c];
  for (int r = 0; r < R; ++r) {
    const uint64_t code = ((uint64_t)codes[(long long)r * n + hd]) >> (3 * pd);
    new_codes[(long long)r * m + c] = (int64_t)code;
    if (keys) keys[(long long)r * m + c] = ((uint64_t)r << code_bits) | code;
  }
  for (int k = 0; k < 3; ++k) new_grid[3 * c + k] = grid[3 * hd + k] >> pd;
  if (new_batch) new_batch[c] = batch ? batch[hd] : 0;
}

// max over each run of X rows (X = proj(feat), [n, C]) -> BN affine -> act   (segment_csr 'max' + norm + act)
// One wave per cluster, four clusters per workgroup, lanes over 4-column groups (C % 4 == 0, 16-byte rows): the
// one-workgroup-per-cluster form launched 15k-90k workgroups of 64-256 threads for runs of 1-8 rows.
__global__ void __launch_bounds__(256) segment_max_affine_act4_kernel(int m, int C, const int* __restrict__ idx_ptr,
                                                                      const int* __restrict__ sorted_idx,
                                                                      const float* __restrict__ X,
                                                                      const float* __restrict__ scale,
                                                                      const float* __restrict__ shift, int act,
                                                                      float* __restrict__ Y) {
  const int c = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= m) return;
  const int beg = __builtin_amdgcn_readfirstlane(idx_ptr[c]), end = __builtin_amdgcn_readfirstlane(idx_ptr[c + 1]);
  for (int g = lane; 4 * g < C; g += 64) {
    float4 v = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    for (int p = beg; p < end; ++p) {
      const int row = __builtin_amdgcn_readfirstlane(sorted_idx[p]);
      const float4 x = *reinterpret_cast<const float4*>(X + (long long)row * C + 4 * g);
      v = make_float4(fmaxf(v.x, x.x), fmaxf(v.y, x.y), fmaxf(v.z, x.z), fmaxf(v.w, x.w));
    }
    float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (scale) o[j] = o[j] * scale[4 * g + j] + shift[4 * g + j];
      if (act == 1) o[j] = 0.5f * o[j] * (1.f + erff(o[j] * 0.70710678118654752f));
    }
    *reinterpret_cast<float4*>(Y + (long long)c * C + 4 * g) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

__global__ void segment_max_affine_act_kernel(int m, int C, const int* __restrict__ idx_ptr,
                                              const int* __restrict__ sorted_idx, const float* __restrict__ X,
                                              const float* __restrict__ scale, const float* __restrict__ shift,
                                              int act, float* __restrict__ Y) {
  const int c = blockIdx.x;
  const int beg = idx_ptr[c], end = idx_ptr[c + 1];
  for (int col = threadIdx.x; col < C; col += blockDim.x) {
    float v = -INFINITY;
    for (int p = beg; p < end; ++p) v = fmaxf(v, X[(long long)sorted_idx[p] * C + col]);
    if (scale) v = v * scale[col] + shift[col];
    if (act == 1) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    Y[(long long)c * C + col] = v;
  }
}

__global__ void segment_mean_kernel(int m, int D, const int* __restrict__ idx_ptr, const int* __restrict__ sorted_idx,
                                    const float* __restrict__ X, float* __restrict__ Y) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= m) return;
  const int beg = idx_ptr[c], end = idx_ptr[c + 1];
  for (int d = 0; d < D; ++d) {
    float s = 0.f;
    for (int p = beg; p < end; ++p) s += X[(long long)sorted_idx[p] * D + d];
    Y[(long long)c * D + d] = s / (float)max(end - beg, 1);
  }
}

// The stage-0 renumbering of a serialized point set by its first serialized order: new point i = old point
// perm[i] (perm = order row 0), so the backbone's stage-0 row gathers follow the serialization.  Codes, orders
// and inverses are re-expressed in the new numbering (order row 0 becomes the identity); grid and coord gathered.
__global__ void __launch_bounds__(256) serialize_permute_kernel(int n, int R, const int* __restrict__ order,
                                                                const int* __restrict__ inverse,
                                                                const int64_t* __restrict__ codes,
                                                                const int* __restrict__ grid,
                                                                const float* __restrict__ coord,
                                                                int64_t* __restrict__ codes_p, int* __restrict__ order_p,
                                                                int* __restrict__ inverse_p, int* __restrict__ grid_p,
                                                                float* __restrict__ coord_p) {
  const int i = (int)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int j = order[i];  // perm[i]: row 0 of order
  for (int r = 0; r < R; ++r) {
    const long long o = (long long)r * n;
    codes_p[o + i] = codes[o + j];
    inverse_p[o + i] = inverse[o + j];
    order_p[o + i] = inverse[order[o + i]];  // the new index of the point at serialized position i of order r
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    grid_p[3ll * i + k] = grid[3ll * j + k];
    coord_p[3ll * i + k] = coord[3ll * j + k];
  }
}

}  // namespace

extern "C" {

// codes[R][n] (int64, batch << 3*depth | code) and keys[R*n] = r << code_bits | code for sfx_sort_pairs_u64.
// order_types: 0 "z", 1 "z-trans", 2 "hilbert", 3 "hilbert-trans".
int sfx_serialize_keys(int n, const int* grid_coord, const int* batch, int depth, int num_orders, int t0, int t1,
                       int t2, int t3, int code_bits, int64_t* codes, uint64_t* keys, void* stream) {
  SFX_REQUIRE(n >= 0 && num_orders >= 1 && num_orders <= 4, "sfx_serialize_keys: bad sizes");
  SFX_REQUIRE(depth >= 1 && depth <= 16, "sfx_serialize_keys: depth must be in [1, 16]");
  SFX_REQUIRE(code_bits + 2 <= 64, "sfx_serialize_keys: code_bits too large");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(grid_coord && codes && keys, "sfx_serialize_keys: null buffer");
  serialize_keys_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(
      n, grid_coord, batch, depth, num_orders, make_int4(t0, t1, t2, t3), code_bits, codes, keys);
  return sfx::check_launch("sfx_serialize_keys");
}

int sfx_serialize_permute(int n, int num_orders, const int* order, const int* inverse, const int64_t* codes,
                          const int* grid, const float* coord, int64_t* codes_p, int* order_p, int* inverse_p,
                          int* grid_p, float* coord_p, void* stream) {
  SFX_REQUIRE(n >= 0 && num_orders >= 1, "sfx_serialize_permute: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(order && inverse && codes && grid && coord && codes_p && order_p && inverse_p && grid_p && coord_p,
              "sfx_serialize_permute: null buffer");
  serialize_permute_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(
      n, num_orders, order, inverse, codes, grid, coord, codes_p, order_p, inverse_p, grid_p, coord_p);
  return sfx::check_launch("sfx_serialize_permute");
}

int sfx_serialize_finalize(int n, int num_orders, const int* sorted_pos, int* order, int* inverse, void* stream) {
  SFX_REQUIRE(n >= 0 && num_orders >= 1, "sfx_serialize_finalize: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(sorted_pos && order && inverse, "sfx_serialize_finalize: null buffer");
  const long long tot = (long long)n * num_orders;
  serialize_finalize_kernel<<<sfx::ceil_div(tot, 256), 256, 0, sfx::as_stream(stream)>>>(n, num_orders, sorted_pos,
                                                                                          order, inverse);
  return sfx::check_launch("sfx_serialize_finalize");
}

int sfx_pool_run_flags(int n, int num_orders, const int* order, const int64_t* codes, int shift, int* flags,
                       void* stream) {
  SFX_REQUIRE(n >= 0 && num_orders >= 1 && shift >= 0 && shift < 64, "sfx_pool_run_flags: bad args");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(order && codes && flags, "sfx_pool_run_flags: null buffer");
  const long long tot = (long long)n * num_orders;
  pool_run_flags_kernel<<<sfx::ceil_div(tot, 256), 256, 0, sfx::as_stream(stream)>>>(n, num_orders, order, codes,
                                                                                     shift, flags);
  return sfx::check_launch("sfx_pool_run_flags");
}

// (ABI v15) counts[k] = number of runs of codes[order[j]] >> shifts[k] along one serialized row (k < nshift <= 8)
int sfx_pool_run_counts(int n, const int* order, const int64_t* codes, const int* shifts, int nshift, int* counts,
                        void* stream) {
  SFX_REQUIRE(n >= 0 && nshift >= 1 && nshift <= 8, "sfx_pool_run_counts: bad args");
  SFX_REQUIRE(shifts && counts, "sfx_pool_run_counts: null buffer");
  RunShifts sh{};
  for (int k = 0; k < nshift; ++k) {
    SFX_REQUIRE(shifts[k] >= 0 && shifts[k] < 64, "sfx_pool_run_counts: shift out of range");
    sh.s[k] = shifts[k];
  }
  hipStream_t st = sfx::as_stream(stream);
  if (hipMemsetAsync(counts, 0, sizeof(int) * (size_t)nshift, st) != hipSuccess)
    return sfx::check_launch("sfx_pool_run_counts (zero)");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(order && codes, "sfx_pool_run_counts: null buffer");
  pool_run_counts_kernel<<<sfx::ceil_div(n, 256), 256, 0, st>>>(n, order, codes, sh, nshift, counts);
  return sfx::check_launch("sfx_pool_run_counts");
}

int sfx_pool_assign_runs(int n, int m, int row0, const int* order, const int* pos, const int* flags, int* cluster,
                         int* idx_ptr, int* head, int* sorted_idx, void* stream) {
  SFX_REQUIRE(n >= 0 && m >= 0 && m <= n && row0 >= 0, "sfx_pool_assign_runs: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(order && pos && flags && cluster && idx_ptr && head && sorted_idx, "sfx_pool_assign_runs: null buffer");
  pool_assign_runs_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, m, row0, order, pos, flags,
                                                                                     cluster, idx_ptr, head,
                                                                                     sorted_idx);
  return sfx::check_launch("sfx_pool_assign_runs");
}

int sfx_pool_reorder(int n, int m, int num_orders, const int* order, const int* pos, const int* flags,
                     const int* cluster, int* new_order, int* new_inverse, void* stream) {
  SFX_REQUIRE(n >= 0 && m >= 0 && m <= n && num_orders >= 1, "sfx_pool_reorder: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(order && pos && flags && cluster && new_order && new_inverse, "sfx_pool_reorder: null buffer");
  const long long tot = (long long)n * num_orders;
  pool_reorder_kernel<<<sfx::ceil_div(tot, 256), 256, 0, sfx::as_stream(stream)>>>(n, m, num_orders, order, pos,
                                                                                   flags, cluster, new_order,
                                                                                   new_inverse);
  return sfx::check_launch("sfx_pool_reorder");
}

int sfx_pool_gather(int m, int n, int num_orders, const int* head, const int64_t* codes, int pooling_depth,
                    const int* grid_coord, const int* batch, int code_bits, int64_t* new_codes, uint64_t* keys,
                    int* new_grid, int* new_batch, void* stream) {
  SFX_REQUIRE(m >= 0 && n >= m && num_orders >= 1 && pooling_depth >= 0, "sfx_pool_gather: bad sizes");
  if (m == 0) return SFX_OK;
  SFX_REQUIRE(head && codes && grid_coord && new_codes && new_grid, "sfx_pool_gather: null buffer");
  pool_gather_kernel<<<sfx::ceil_div(m, 256), 256, 0, sfx::as_stream(stream)>>>(
      m, n, num_orders, head, codes, pooling_depth, grid_coord, batch, nullptr, code_bits, new_codes, keys, new_grid,
      new_batch);
  return sfx::check_launch("sfx_pool_gather");
}

int sfx_segment_max_affine_act(int m, int C, const int* idx_ptr, const int* sorted_idx, const float* X,
                               const float* scale, const float* shift, int act, float* Y, void* stream) {
  SFX_REQUIRE(m >= 0 && C > 0 && (act == 0 || act == 1), "sfx_segment_max_affine_act: bad args");
  if (m == 0) return SFX_OK;
  SFX_REQUIRE(idx_ptr && sorted_idx && X && Y, "sfx_segment_max_affine_act: null buffer");
  static const bool v4 = !(getenv("SFX_SEGMAX4") && !strcmp(getenv("SFX_SEGMAX4"), "0"));
  if (v4 && C % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (reinterpret_cast<uintptr_t>(Y) & 15) == 0) {
    segment_max_affine_act4_kernel<<<sfx::ceil_div(m, 4), 256, 0, sfx::as_stream(stream)>>>(
        m, C, idx_ptr, sorted_idx, X, scale, shift, act, Y);
    return sfx::check_launch("sfx_segment_max_affine_act");
  }
  const int threads = C >= 256 ? 256 : (C >= 128 ? 128 : 64);
  segment_max_affine_act_kernel<<<m, threads, 0, sfx::as_stream(stream)>>>(m, C, idx_ptr, sorted_idx, X, scale,
                                                                          shift, act, Y);
  return sfx::check_launch("sfx_segment_max_affine_act");
}

int sfx_segment_mean(int m, int D, const int* idx_ptr, const int* sorted_idx, const float* X, float* Y,
                     void* stream) {
  SFX_REQUIRE(m >= 0 && D > 0, "sfx_segment_mean: bad args");
  if (m == 0) return SFX_OK;
  SFX_REQUIRE(idx_ptr && sorted_idx && X && Y, "sfx_segment_mean: null buffer");
  segment_mean_kernel<<<sfx::ceil_div(m, 256), 256, 0, sfx::as_stream(stream)>>>(m, D, idx_ptr, sorted_idx, X, Y);
  return sfx::check_launch("sfx_segment_mean");
}

}  // extern "C"
