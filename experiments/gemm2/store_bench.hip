// Store-pattern microbenchmark (diagnostic, not product): a [M][N] fp32 matrix written by 256 persistent
// 512-thread workgroups in 256 x 128 tiles, each wave a 64 x 64 block as four 32 x 32 accumulator blocks, in the
// store shapes a 32x32x16 MFMA epilogue can produce:
//   0  lane = row, 16 B per lane (4 consecutive columns): 32 rows x 32 B per instruction      (gemm2 swapped)
//   1  lane = column, 4 B per lane: 2 rows x 128 B per instruction                             (gemm.hip)
//   2  16 lanes per row, 16 B per lane: 4 rows x 256 B per instruction (needs a transpose)      (ideal)
// build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/store_bench.hip -o tools/store_bench.so
#include <hip/hip_runtime.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int PAT>
__global__ void __launch_bounds__(512, 1) store_kernel(float* Y, int M, int N, int tiles_n, int total) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const int h = lane >> 5, r32 = lane & 31;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(Y, (short)0, 0x7ffffff0, 0x00020000);
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    const int m0 = (t / tiles_n) * 256 + wm * 64, n0 = (t % tiles_n) * 128 + wn * 64;
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
      const int bm = m0 + (blk >> 1) * 32, bn = n0 + (blk & 1) * 32;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (PAT == 0) {
          const int m = bm + r32, n = bn + 8 * i + 4 * h;
          const u32x4 v = {(unsigned)m, (unsigned)n, 1u, 2u};
          __builtin_amdgcn_raw_buffer_store_b128(v, r, (m < M && n < N) ? (unsigned)(m * N + n) * 4u : 0x7ffffff0u, 0, 0);
        } else if (PAT == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int m = bm + j + 8 * i + 4 * h, n = bn + r32;
            __builtin_amdgcn_raw_buffer_store_b32((unsigned)m, r, (m < M && n < N) ? (unsigned)(m * N + n) * 4u : 0x7ffffff0u, 0, 0);
          }
        } else {
          // 16 lanes per 64-column row: lane -> row (lane >> 4) + 4 i + 16 (blk & 1)... of the wave's 64 x 64 block
          const int m = m0 + (blk * 4 + i) * 4 + (lane >> 4), n = n0 + 4 * (lane & 15);
          const u32x4 v = {(unsigned)m, (unsigned)n, 1u, 2u};
          __builtin_amdgcn_raw_buffer_store_b128(v, r, (m < M && n < N) ? (unsigned)(m * N + n) * 4u : 0x7ffffff0u, 0, 0);
        }
      }
    }
  }
}

extern "C" int store_bench(int pat, float* Y, int M, int N, void* stream) {
  const int tiles_n = (N + 127) / 128, total = ((M + 255) / 256) * tiles_n;
  const int grid = total < 256 ? total : 256;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (pat == 0) store_kernel<0><<<grid, 512, 0, s>>>(Y, M, N, tiles_n, total);
  else if (pat == 1) store_kernel<1><<<grid, 512, 0, s>>>(Y, M, N, tiles_n, total);
  else store_kernel<2><<<grid, 512, 0, s>>>(Y, M, N, tiles_n, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
