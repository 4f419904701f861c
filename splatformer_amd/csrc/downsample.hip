// Point-cloud downsampling experiments of the fork (reference models/pcd_downsampling_methods.py, selected by
// FeaturePredictor additional_info["downsample"], reference models/feature_predictor.py:159-196):
//   * sfx_voxel_keys -- voxel ids of voxel_downsample (:86-130): floor(p / voxel_size) in fp32 with the
//     correctly rounded division (__fdiv_rn) torch's CPU true_divide computes -- the goldens were captured on the
//     CPU; a CUDA run of the reference may compute p * (1 / voxel_size) and floor a boundary point into the
//     neighbouring voxel, so parity against the reference's GPU run is unpinned; the int32 hash
//     x * 1e6 + y * 1e3 + z (int32 wrap-around as torch computes it), biased to an unsigned sort key; the
//     unique / inverse / mean steps reuse the radix sort, run-flag, scan and segment-mean kernels.
//   * sfx_nn1 -- 1-nearest neighbour of every query among the reference points (sklearn NearestNeighbors in
//     fps_knn_downsample :45-48 and knn_map_back :182-198): brute force over LDS tiles of the reference set,
//     float64 squared distances of the float32 coordinates (sklearn computes in float64), lowest index on ties.
//   * sfx_fps -- furthest_point_sampling (:8-26): one workgroup iterating the M picks, fp32 squared distances
//     without contraction (torch's elementwise square + sum), running minimum, arg-max with the lowest index.
#include "common.h"

namespace {

__global__ void voxel_keys_kernel(int n, const float* __restrict__ pts, long long ld, float vs,
                                  unsigned long long* __restrict__ keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = pts + (long long)i * ld;
  const int vx = (int)floorf(__fdiv_rn(p[0], vs));
  const int vy = (int)floorf(__fdiv_rn(p[1], vs));
  const int vz = (int)floorf(__fdiv_rn(p[2], vs));
  const unsigned id = (unsigned)vx * 1000000u + (unsigned)vy * 1000u + (unsigned)vz;  // int32 wrap-around
  keys[i] = (unsigned long long)(id ^ 0x80000000u);  // signed order as unsigned
}

constexpr int NN_TILE = 1024;

__global__ void __launch_bounds__(256) nn1_kernel(int n, int m, const float* __restrict__ q,
                                                  const float* __restrict__ r, int* __restrict__ out) {
  __shared__ float rs[NN_TILE * 3];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = i < n;
  const double qx = ok ? (double)q[3ll * i] : 0.0, qy = ok ? (double)q[3ll * i + 1] : 0.0,
               qz = ok ? (double)q[3ll * i + 2] : 0.0;
  double best = __builtin_inf();
  int bi = 0;
  for (int t0 = 0; t0 < m; t0 += NN_TILE) {
    const int cnt = min(NN_TILE, m - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < cnt * 3; e += blockDim.x) rs[e] = r[3ll * t0 + e];
    __syncthreads();
    for (int j = 0; j < cnt; ++j) {
      const double dx = qx - (double)rs[3 * j], dy = qy - (double)rs[3 * j + 1], dz = qz - (double)rs[3 * j + 2];
      const double d = __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz));
      if (d < best) {
        best = d;
        bi = t0 + j;
      }
    }
  }
  if (ok) out[i] = bi;
}

constexpr int FPS_THREADS = 1024;

__global__ void __launch_bounds__(FPS_THREADS) fps_kernel(int n, int m, const float* __restrict__ xyz, int start,
                                                          int* __restrict__ out, float* __restrict__ dist) {
  __shared__ float wv[FPS_THREADS / 64];
  __shared__ int wi[FPS_THREADS / 64];
  __shared__ int far_s;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < n; i += FPS_THREADS) dist[i] = 1e10f;
  int far = start;
  for (int it = 0; it < m; ++it) {  // every thread runs all m picks: the exit is uniform
    if (tid == 0) out[it] = far;
    const float cx = xyz[3ll * far], cy = xyz[3ll * far + 1], cz = xyz[3ll * far + 2];
    float bv = -1.f;
    int bidx = 0x7fffffff;
    for (int i = tid; i < n; i += FPS_THREADS) {
      const float dx = __fsub_rn(xyz[3ll * i], cx), dy = __fsub_rn(xyz[3ll * i + 1], cy),
                  dz = __fsub_rn(xyz[3ll * i + 2], cz);
      const float d = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
      float cur = dist[i];
      if (d < cur) {
        cur = d;
        dist[i] = d;
      }
      if (cur > bv) {  // strided ascending i: the first maximum of this thread
        bv = cur;
        bidx = i;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bidx, o, 64);
      if (ov > bv || (ov == bv && oi < bidx)) {
        bv = ov;
        bidx = oi;
      }
    }
    if (lane == 0) {
      wv[wid] = bv;
      wi[wid] = bidx;
    }
    __syncthreads();
    if (tid == 0) {
      float v = wv[0];
      int x = wi[0];
      for (int w = 1; w < FPS_THREADS / 64; ++w)
        if (wv[w] > v || (wv[w] == v && wi[w] < x)) {
          v = wv[w];
          x = wi[w];
        }
      far_s = x;
    }
    __syncthreads();
    far = far_s;
  }
}

}  // namespace

extern "C" {

int sfx_voxel_keys(int n, const float* points, long long ld, float voxel_size, unsigned long long* keys,
                   void* stream) {
  SFX_REQUIRE(n >= 0 && ld >= 3 && voxel_size > 0.f, "sfx_voxel_keys: bad args");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(points && keys, "sfx_voxel_keys: null buffer");
  voxel_keys_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, points, ld, voxel_size, keys);
  return sfx::check_launch("sfx_voxel_keys");
}

int sfx_nn1(int n, int m, const float* queries, const float* refs, int* out, void* stream) {
  SFX_REQUIRE(n >= 0 && m >= 0, "sfx_nn1: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(m > 0, "sfx_nn1: empty reference set");
  SFX_REQUIRE(queries && refs && out, "sfx_nn1: null buffer");
  nn1_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, m, queries, refs, out);
  return sfx::check_launch("sfx_nn1");
}

int sfx_fps(int n, int m, const float* xyz, int start, int* out, float* dist_ws, void* stream) {
  SFX_REQUIRE(n >= 0 && m >= 0 && m <= n, "sfx_fps: bad sizes");
  if (m == 0) return SFX_OK;
  SFX_REQUIRE(start >= 0 && start < n, "sfx_fps: start out of range");
  SFX_REQUIRE(xyz && out && dist_ws, "sfx_fps: null buffer");
  fps_kernel<<<1, FPS_THREADS, 0, sfx::as_stream(stream)>>>(n, m, xyz, start, out, dist_ws);
  return sfx::check_launch("sfx_fps");
}

}  // extern "C"
