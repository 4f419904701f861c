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

__global__ void subm_query_kernel(int n, const int* __restrict__ grid, const int* __restrict__ batch,
                                  const unsigned long long* __restrict__ keys, const int* __restrict__ vals,
                                  int log2cap, int* __restrict__ nbr) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 27ll * n) return;
  const int i = (int)(t / 27), k = (int)(t - (long long)i * 27);
  const int dx = k / 9 - 1, dy = (k / 3) % 3 - 1, dz = k % 3 - 1;
  const int x = grid[3 * i] + dx, y = grid[3 * i + 1] + dy, z = grid[3 * i + 2] + dz;
  int out = -1;
  if (x >= 0 && y >= 0 && z >= 0) {
    const unsigned long long key = pack(batch ? batch[i] : 0, x, y, z);
    const unsigned mask = (1u << log2cap) - 1u;
    unsigned s = slot_of(key, log2cap);
    while (true) {
      const unsigned long long kk = keys[s];
      if (kk == key) {
        out = vals[s];
        break;
      }
      if (kk == EMPTY) break;
      s = (s + 1) & mask;
    }
  }
  nbr[t] = out;
}

}  // namespace

extern "C" {

int sfx_subm_table_log2(int n) {
  int l = 4;
  while ((1ll << l) < 2ll * (n > 0 ? n : 1)) ++l;
  return l;
}

// table_keys: 2^log2cap u64, table_vals: 2^log2cap i32 (both scratch); nbr: [n][27] i32
int sfx_subm_neighbors(int n, const int* grid_coord, const int* batch, int log2cap, unsigned long long* table_keys,
                       int* table_vals, int* nbr, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_subm_neighbors: n < 0");
  SFX_REQUIRE(log2cap >= 4 && log2cap <= 31 && (1ll << log2cap) >= 2ll * n, "sfx_subm_neighbors: table too small");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(grid_coord && table_keys && table_vals && nbr, "sfx_subm_neighbors: null buffer");
  hipStream_t st = sfx::as_stream(stream);
  const size_t cap = (size_t)1 << log2cap;
  hipMemsetAsync(table_keys, 0xff, cap * sizeof(unsigned long long), st);
  hipMemsetAsync(table_vals, 0x7f, cap * sizeof(int), st);
  subm_insert_kernel<<<sfx::ceil_div(n, 256), 256, 0, st>>>(n, grid_coord, batch, table_keys, table_vals, log2cap);
  subm_query_kernel<<<sfx::ceil_div(27ll * n, 256), 256, 0, st>>>(n, grid_coord, batch, table_keys, table_vals,
                                                                  log2cap, nbr);
  return sfx::check_launch("sfx_subm_neighbors");
}

}  // extern "C"
