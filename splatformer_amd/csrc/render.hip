// Gaussian render path: SH evaluation, EWA projection, tile binning and
// tile-local front-to-back alpha compositing (forward + backward).
//
// Semantics follow gsplat v0.1.11 (the version pinned at reference
// README.md:27 and called from reference utils/gs_utils.py:78, :82-95, :96-109);
// see SURVEY.md Appendix A.2 and oracle/gsplat_ref.py for the restatement.
// Layout: AoS float records exactly as the gsplat tensors ([N,3] means, [N,4]
// quats (w,x,y,z), [N,2] xys, [N,3] conics ...), so the drop-in shim can hand
// torch tensors straight through.  One workgroup of bw*bw lanes (4 waves at
// bw=16) per 16x16 tile; per-batch Gaussian records staged in LDS.
#include <climits>

#include "common.h"

namespace {

__constant__ float SH_C0 = 0.28209479177387814f;
__constant__ float SH_C1 = 0.4886025119029199f;
__constant__ float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
__constant__ float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};
__constant__ float SH_C4[9] = {2.5033429417967046f,  -1.7701307697799304f, 0.9461746957575601f,
                               -0.6690465435572892f, 0.10578554691520431f, -0.6690465435572892f,
                               0.47308734787878004f, -1.7701307697799304f, 0.6258357354491761f};

// ---- spherical harmonics ---------------------------------------------------
// basis values for degree <= 4 into b[0..(d+1)^2)
__device__ __forceinline__ void sh_basis(int degree, float x, float y, float z, float* b) {
  b[0] = SH_C0;
  if (degree < 1) return;
  b[1] = -SH_C1 * y;
  b[2] = SH_C1 * z;
  b[3] = -SH_C1 * x;
  if (degree < 2) return;
  const float xx = x * x, xy = x * y, xz = x * z, yy = y * y, yz = y * z, zz = z * z;
  b[4] = SH_C2[0] * xy;
  b[5] = SH_C2[1] * yz;
  b[6] = SH_C2[2] * (2.f * zz - xx - yy);
  b[7] = SH_C2[3] * xz;
  b[8] = SH_C2[4] * (xx - yy);
  if (degree < 3) return;
  b[9] = SH_C3[0] * y * (3.f * xx - yy);
  b[10] = SH_C3[1] * xy * z;
  b[11] = SH_C3[2] * y * (4.f * zz - xx - yy);
  b[12] = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
  b[13] = SH_C3[4] * x * (4.f * zz - xx - yy);
  b[14] = SH_C3[5] * z * (xx - yy);
  b[15] = SH_C3[6] * x * (xx - 3.f * yy);
  if (degree < 4) return;
  b[16] = SH_C4[0] * xy * (xx - yy);
  b[17] = SH_C4[1] * yz * (3.f * xx - yy);
  b[18] = SH_C4[2] * xy * (7.f * zz - 1.f);
  b[19] = SH_C4[3] * yz * (7.f * zz - 3.f);
  b[20] = SH_C4[4] * (zz * (35.f * zz - 30.f) + 3.f);
  b[21] = SH_C4[5] * xz * (7.f * zz - 3.f);
  b[22] = SH_C4[6] * (xx - yy) * (7.f * zz - 1.f);
  b[23] = SH_C4[7] * xz * (xx - 3.f * yy);
  b[24] = SH_C4[8] * (xx * (xx - 3.f * yy) - yy * (3.f * xx - yy));
}

__global__ void sh_fwd_kernel(int n, int num_bases, int degrees_to_use, const float* __restrict__ viewdirs,
                              const float* __restrict__ coeffs, float* __restrict__ colors) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* c = coeffs + (size_t)i * num_bases * 3;
  float x = 0.f, y = 0.f, z = 0.f;
  if (degrees_to_use >= 1) {
    const float vx = viewdirs[3 * i], vy = viewdirs[3 * i + 1], vz = viewdirs[3 * i + 2];
    const float nrm = sqrtf(vx * vx + vy * vy + vz * vz);
    x = vx / nrm; y = vy / nrm; z = vz / nrm;
  }
  // grouping follows gsplat sh_coeffs_to_color: one bracketed sum per degree
  const float xx = x * x, xy = x * y, xz = x * z, yy = y * y, yz = y * z, zz = z * z;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    float acc = SH_C0 * c[ch];
    if (degrees_to_use >= 1) {
      acc += SH_C1 * (-y * c[3 + ch] + z * c[6 + ch] - x * c[9 + ch]);
      if (degrees_to_use >= 2) {
        acc += (SH_C2[0] * xy * c[12 + ch] + SH_C2[1] * yz * c[15 + ch] + SH_C2[2] * (2.f * zz - xx - yy) * c[18 + ch] +
                SH_C2[3] * xz * c[21 + ch] + SH_C2[4] * (xx - yy) * c[24 + ch]);
        if (degrees_to_use >= 3) {
          acc += (SH_C3[0] * y * (3.f * xx - yy) * c[27 + ch] + SH_C3[1] * xy * z * c[30 + ch] +
                  SH_C3[2] * y * (4.f * zz - xx - yy) * c[33 + ch] +
                  SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy) * c[36 + ch] +
                  SH_C3[4] * x * (4.f * zz - xx - yy) * c[39 + ch] + SH_C3[5] * z * (xx - yy) * c[42 + ch] +
                  SH_C3[6] * x * (xx - 3.f * yy) * c[45 + ch]);
          if (degrees_to_use >= 4) {
            acc += (SH_C4[0] * xy * (xx - yy) * c[48 + ch] + SH_C4[1] * yz * (3.f * xx - yy) * c[51 + ch] +
                    SH_C4[2] * xy * (7.f * zz - 1.f) * c[54 + ch] + SH_C4[3] * yz * (7.f * zz - 3.f) * c[57 + ch] +
                    SH_C4[4] * (zz * (35.f * zz - 30.f) + 3.f) * c[60 + ch] +
                    SH_C4[5] * xz * (7.f * zz - 3.f) * c[63 + ch] +
                    SH_C4[6] * (xx - yy) * (7.f * zz - 1.f) * c[66 + ch] +
                    SH_C4[7] * xz * (xx - 3.f * yy) * c[69 + ch] +
                    SH_C4[8] * (xx * (xx - 3.f * yy) - yy * (3.f * xx - yy)) * c[72 + ch]);
          }
        }
      }
    }
    colors[3 * i + ch] = acc;
  }
}

__global__ void sh_bwd_kernel(int n, int num_bases, int degrees_to_use, const float* __restrict__ viewdirs,
                              const float* __restrict__ v_colors, float* __restrict__ v_coeffs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float b[25];
  float x = 0.f, y = 0.f, z = 0.f;
  if (degrees_to_use >= 1) {
    const float vx = viewdirs[3 * i], vy = viewdirs[3 * i + 1], vz = viewdirs[3 * i + 2];
    const float nrm = sqrtf(vx * vx + vy * vy + vz * vz);
    x = vx / nrm; y = vy / nrm; z = vz / nrm;
  }
  sh_basis(degrees_to_use, x, y, z, b);
  const int nb = (degrees_to_use + 1) * (degrees_to_use + 1);
  float* vc = v_coeffs + (size_t)i * num_bases * 3;
  const float g0 = v_colors[3 * i], g1 = v_colors[3 * i + 1], g2 = v_colors[3 * i + 2];
  for (int k = 0; k < num_bases; ++k) {
    const float bk = k < nb ? b[k] : 0.f;
    vc[3 * k + 0] = bk * g0;
    vc[3 * k + 1] = bk * g1;
    vc[3 * k + 2] = bk * g2;
  }
}

// ---- projection -------------------------------------------------------------
struct M3 {  // row-major 3x3
  float m[3][3];
};

// Canonical arithmetic of the projection (oracle/gsplat_ref.py project_gaussians): every fp32 product and sum
// rounded on its own (contraction off in these bodies; the library builds with -ffp-contract=fast-honor-pragmas), sums of
// products left to right, correctly rounded division and sqrt (1/sqrt instead of an approximate rsqrt) --
// radii, tile counts, intersection keys and the projected floats are bit-identical to the oracle.
__device__ __forceinline__ M3 quat_to_rotmat(float qw, float qx, float qy, float qz) {
#pragma clang fp contract(off)
  const float s = 1.f / sqrtf(((qw * qw + qx * qx) + qy * qy) + qz * qz);
  const float w = qw * s, x = qx * s, y = qy * s, z = qz * s;
  M3 R;
  R.m[0][0] = 1.f - 2.f * (y * y + z * z);
  R.m[0][1] = 2.f * (x * y - w * z);
  R.m[0][2] = 2.f * (x * z + w * y);
  R.m[1][0] = 2.f * (x * y + w * z);
  R.m[1][1] = 1.f - 2.f * (x * x + z * z);
  R.m[1][2] = 2.f * (y * z - w * x);
  R.m[2][0] = 2.f * (x * z - w * y);
  R.m[2][1] = 2.f * (y * z + w * x);
  R.m[2][2] = 1.f - 2.f * (x * x + y * y);
  return R;
}

__device__ __forceinline__ void get_tile_bbox(float cx, float cy, float radius, int tiles_x, int tiles_y, int bw,
                                              int& x0, int& y0, int& x1, int& y1) {
  // gsplat get_tile_bbox/get_bbox: (int) truncation, clamp to [0, tiles]
  const float tcx = cx / (float)bw, tcy = cy / (float)bw;
  const float tr = radius / (float)bw;
  x0 = min(max(0, (int)(tcx - tr)), tiles_x);
  x1 = min(max(0, (int)(tcx + tr + 1.f)), tiles_x);
  y0 = min(max(0, (int)(tcy - tr)), tiles_y);
  y1 = min(max(0, (int)(tcy + tr + 1.f)), tiles_y);
}

// One Gaussian of project_gaussians_forward_kernel.  Writes every output
// (zeros for culled points, as gsplat's torch::zeros-initialised buffers);
// comp / cov3d may be null.
__device__ __forceinline__ void project_point(int i, float px, float py, float pz, float sc0, float sc1, float sc2,
                                              float qw, float qx, float qy, float qz, float glob_scale,
                                              const float* vm, float fx, float fy, float cx, float cy, int img_h,
                                              int img_w, int bw, float clip_thresh, float* __restrict__ xys,
                                              float* __restrict__ depths, int* __restrict__ radii,
                                              float* __restrict__ conics, float* __restrict__ comp,
                                              int* __restrict__ num_tiles_hit, float* __restrict__ cov3d) {
#pragma clang fp contract(off)
  const int tiles_x = (img_w + bw - 1) / bw, tiles_y = (img_h + bw - 1) / bw;
  float o_xy0 = 0.f, o_xy1 = 0.f, o_depth = 0.f, o_comp = 0.f;
  float o_con0 = 0.f, o_con1 = 0.f, o_con2 = 0.f;
  float cv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int o_radius = 0, o_tiles = 0;
  const float tx = vm[0] * px + vm[1] * py + vm[2] * pz + vm[3];
  const float ty = vm[4] * px + vm[5] * py + vm[6] * pz + vm[7];
  const float tz = vm[8] * px + vm[9] * py + vm[10] * pz + vm[11];
  do {
    if (tz <= clip_thresh) break;
    // cov3d = R S S^T R^T
    const M3 R = quat_to_rotmat(qw, qx, qy, qz);
    const float s0 = glob_scale * sc0, s1 = glob_scale * sc1, s2 = glob_scale * sc2;
    float M[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      M[r][0] = R.m[r][0] * s0;
      M[r][1] = R.m[r][1] * s1;
      M[r][2] = R.m[r][2] * s2;
    }
    float V[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) V[r][c] = (M[r][0] * M[c][0] + M[r][1] * M[c][1]) + M[r][2] * M[c][2];
    cv[0] = V[0][0]; cv[1] = V[0][1]; cv[2] = V[0][2];
    cv[3] = V[1][1]; cv[4] = V[1][2]; cv[5] = V[2][2];
    // EWA: t clamped to 1.3 tan_fov frustum
    // gsplat: tan_fov = 0.5 * img_size / f in double, stored as float; lim = 1.3f * tan_fov in float
    const float tan_fovx = (float)(0.5 * (double)img_w / (double)fx);
    const float tan_fovy = (float)(0.5 * (double)img_h / (double)fy);
    const float lim_x = 1.3f * tan_fovx, lim_y = 1.3f * tan_fovy;
    const float ctx = tz * fminf(lim_x, fmaxf(-lim_x, tx / tz));
    const float cty = tz * fminf(lim_y, fmaxf(-lim_y, ty / tz));
    const float rz = 1.f / tz, rz2 = rz * rz;
    // J (2x3): [[fx rz, 0, -fx tx rz2], [0, fy rz, -fy ty rz2]]
    const float j00 = fx * rz, j02 = -fx * ctx * rz2, j11 = fy * rz, j12 = -fy * cty * rz2;
    // T = J W, W = viewmat[:3,:3] (row-major)
    float T0[3], T1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      T0[c] = j00 * vm[0 + c] + j02 * vm[8 + c];
      T1[c] = j11 * vm[4 + c] + j12 * vm[8 + c];
    }
    // cov2d = T V T^T
    float TV0[3], TV1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      TV0[c] = (T0[0] * V[0][c] + T0[1] * V[1][c]) + T0[2] * V[2][c];
      TV1[c] = (T1[0] * V[0][c] + T1[1] * V[1][c]) + T1[2] * V[2][c];
    }
    const float c00 = (TV0[0] * T0[0] + TV0[1] * T0[1]) + TV0[2] * T0[2];
    const float c01 = (TV0[0] * T1[0] + TV0[1] * T1[1]) + TV0[2] * T1[2];
    const float c11 = (TV1[0] * T1[0] + TV1[1] * T1[1]) + TV1[2] * T1[2];
    const float det_orig = c00 * c11 - c01 * c01;
    const float a = c00 + 0.3f, b = c01, c = c11 + 0.3f;
    const float det_blur = a * c - b * b;
    const float compv = sqrtf(fmaxf(0.f, det_orig / det_blur));
    // conic + radius (compute_cov2d_bounds)
    const float det = det_blur;
    if (det == 0.f) break;
    const float inv_det = 1.f / det;
    o_con0 = c * inv_det;
    o_con1 = -b * inv_det;
    o_con2 = a * inv_det;
    const float mid = 0.5f * (a + c);
    const float lam1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float lam2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float radius = ceilf(3.f * sqrtf(fmaxf(lam1, lam2)));
    // center (project_pix)
    const float rw = 1.f / (tz + 1e-6f);
    const float cxp = tx * rw * fx + cx, cyp = ty * rw * fy + cy;
    int x0, y0, x1, y1;
    get_tile_bbox(cxp, cyp, radius, tiles_x, tiles_y, bw, x0, y0, x1, y1);
    const int area = (x1 - x0) * (y1 - y0);
    if (area <= 0) break;
    o_tiles = area;
    o_depth = tz;
    o_radius = (int)radius;
    o_xy0 = cxp;
    o_xy1 = cyp;
    o_comp = compv;
  } while (0);

  xys[2 * i] = o_xy0;
  xys[2 * i + 1] = o_xy1;
  depths[i] = o_depth;
  radii[i] = o_radius;
  conics[3 * i] = o_con0;
  conics[3 * i + 1] = o_con1;
  conics[3 * i + 2] = o_con2;
  if (comp) comp[i] = o_comp;
  num_tiles_hit[i] = o_tiles;
  if (cov3d)
#pragma unroll
    for (int k = 0; k < 6; ++k) cov3d[6 * i + k] = cv[k];
}

__global__ void project_fwd_kernel(int n, const float* __restrict__ means, const float* __restrict__ scales,
                                   float glob_scale, const float* __restrict__ quats, const float* __restrict__ viewmat,
                                   float fx, float fy, float cx, float cy, int img_h, int img_w, int bw,
                                   float clip_thresh, float* __restrict__ xys, float* __restrict__ depths,
                                   int* __restrict__ radii, float* __restrict__ conics, float* __restrict__ comp,
                                   int* __restrict__ num_tiles_hit, float* __restrict__ cov3d) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float vm[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) vm[k] = viewmat[k];
  project_point(i, means[3 * i], means[3 * i + 1], means[3 * i + 2], scales[3 * i], scales[3 * i + 1],
                scales[3 * i + 2], quats[4 * i], quats[4 * i + 1], quats[4 * i + 2], quats[4 * i + 3], glob_scale, vm,
                fx, fy, cx, cy, img_h, img_w, bw, clip_thresh, xys, depths, radii, conics, comp, num_tiles_hit,
                cov3d);
}

// Fused eval-path render prep + SH + projection (reference utils/gs_utils.py:32-95
// in one pass over the Gaussian records): viewmat from camera_to_world with the
// diag(1,-1,-1) flip, scales = exp, quats / ||q|| (NaN -> (0,0,0,1)),
// opacity = sigmoid, SH colours (+0.5, clamp >= 0; sigmoid(dc) at degree 0),
// then project_gaussians with glob_scale 1.  Block 0 lane 0 also stores the
// 3x4 viewmat for the caller.
struct PrepStrides {
  long long means, scales, quats, opac, dc, rest;
};

// One thread per Gaussian, all views in a loop: the Gaussian's parameters (up to 75 SH floats) are read once into
// registers and its view-independent terms (exp scales, normalised quaternion, sigmoid opacity -- fp64 exps) computed
// once, instead of once per (Gaussian, view) thread re-reading them (config E: 9 views x 500k x 59 floats).  The
// per-view arithmetic is unchanged expression for expression (bit-identical outputs).
template <int DEG>
__global__ void __launch_bounds__(256) render_prep_project_kernel(
    int n, int nviews, const float* __restrict__ means, const float* __restrict__ log_scales,
    const float* __restrict__ quats_raw, const float* __restrict__ opac_logit, const float* __restrict__ dc,
    const float* __restrict__ rest, PrepStrides ld, const float* __restrict__ c2ws, float fx, float fy, float cx,
    float cy, int img_h, int img_w, int bw, float* __restrict__ viewmat_out, float* __restrict__ rgbs,
    float* __restrict__ opac, float* __restrict__ xys, float* __restrict__ depths, int* __restrict__ radii,
    float* __restrict__ conics, int* __restrict__ num_tiles_hit, float4* __restrict__ rec) {
  // canonical glue arithmetic (oracle/render_ref.py glue_args(canonical=True)): exp / sigmoid in double rounded
  // once, norms as left-to-right sums with a correctly rounded sqrt, no contraction
#pragma clang fp contract(off)
  constexpr int NB = (DEG + 1) * (DEG + 1);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  // camera v: R = c2w[:3,:3] diag(1,-1,-1); viewmat = [R^T | -R^T t]
  auto camera = [&](int v, float (&t)[3], float (&vm)[12]) {
    const float* c2w = c2ws + 16 * v;
    float R[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R[r][0] = c2w[4 * r + 0];
      R[r][1] = -c2w[4 * r + 1];
      R[r][2] = -c2w[4 * r + 2];
      t[r] = c2w[4 * r + 3];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) vm[4 * r + c] = R[c][r];
      vm[4 * r + 3] = -((R[0][r] * t[0] + R[1][r] * t[1]) + R[2][r] * t[2]);
    }
  };
  if (i == 0 && viewmat_out) {
    float t[3], vm[12];
    camera(0, t, vm);
#pragma unroll
    for (int k = 0; k < 12; ++k) viewmat_out[k] = vm[k];
  }
  if (i >= n) return;
  const float* mp = means + i * ld.means;
  const float* sp = log_scales + i * ld.scales;
  const float* qp = quats_raw + i * ld.quats;
  const float* dcp = dc + i * ld.dc;
  const float px = mp[0], py = mp[1], pz = mp[2];
  const float sc0 = (float)exp((double)sp[0]), sc1 = (float)exp((double)sp[1]), sc2 = (float)exp((double)sp[2]);
  float q0 = qp[0], q1 = qp[1], q2 = qp[2], q3 = qp[3];
  const float qn = sqrtf(((q0 * q0 + q1 * q1) + q2 * q2) + q3 * q3);
  q0 /= qn; q1 /= qn; q2 /= qn; q3 /= qn;
  if (isnan(q0) || isnan(q1) || isnan(q2) || isnan(q3)) {
    q0 = 0.f; q1 = 0.f; q2 = 0.f; q3 = 1.f;
  }
  const float op = (float)(1.0 / (1.0 + exp(-(double)opac_logit[i * ld.opac])));
  float d0[3];
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) d0[ch] = dcp[ch];
  float c[3 * NB];  // c[3*k + ch] for k >= 1 (the rest coefficients), registers
#pragma unroll
  for (int k = 3; k < 3 * NB; ++k) c[k] = rest[i * ld.rest + (k - 3)];
  float rgb0[3];
  if constexpr (DEG == 0) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) rgb0[ch] = (float)(1.0 / (1.0 + exp(-(double)d0[ch])));
  }
  for (int v = 0; v < nviews; ++v) {
    float t[3], vm[12];
    camera(v, t, vm);
    const long long o = (long long)v * n;
    opac[o + i] = op;
    if constexpr (DEG == 0) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) rgbs[3 * (o + i) + ch] = rgb0[ch];
    } else {
      float vx = px - t[0], vy = py - t[1], vz = pz - t[2];
      const float vn = sqrtf((vx * vx + vy * vy) + vz * vz);
      if (vn == 0.f) {  // reference draws a random direction here (gs_utils.py:72-76); we use +z
        vx = 0.f; vy = 0.f; vz = 1.f;
      } else {
        vx /= vn; vy /= vn; vz /= vn;
      }
      const float nrm = sqrtf(vx * vx + vy * vy + vz * vz);
      const float x = vx / nrm, y = vy / nrm, z = vz / nrm;
      const float xx = x * x, xy = x * y, xz = x * z, yy = y * y, yz = y * z, zz = z * z;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        float acc = SH_C0 * d0[ch];
        acc += SH_C1 * (-y * c[3 + ch] + z * c[6 + ch] - x * c[9 + ch]);
        if constexpr (DEG >= 2) {
          acc += (SH_C2[0] * xy * c[12 + ch] + SH_C2[1] * yz * c[15 + ch] + SH_C2[2] * (2.f * zz - xx - yy) * c[18 + ch] +
                  SH_C2[3] * xz * c[21 + ch] + SH_C2[4] * (xx - yy) * c[24 + ch]);
          if constexpr (DEG >= 3) {
            acc += (SH_C3[0] * y * (3.f * xx - yy) * c[27 + ch] + SH_C3[1] * xy * z * c[30 + ch] +
                    SH_C3[2] * y * (4.f * zz - xx - yy) * c[33 + ch] +
                    SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy) * c[36 + ch] +
                    SH_C3[4] * x * (4.f * zz - xx - yy) * c[39 + ch] + SH_C3[5] * z * (xx - yy) * c[42 + ch] +
                    SH_C3[6] * x * (xx - 3.f * yy) * c[45 + ch]);
            if constexpr (DEG >= 4) {
              acc += (SH_C4[0] * xy * (xx - yy) * c[48 + ch] + SH_C4[1] * yz * (3.f * xx - yy) * c[51 + ch] +
                      SH_C4[2] * xy * (7.f * zz - 1.f) * c[54 + ch] + SH_C4[3] * yz * (7.f * zz - 3.f) * c[57 + ch] +
                      SH_C4[4] * (zz * (35.f * zz - 30.f) + 3.f) * c[60 + ch] +
                      SH_C4[5] * xz * (7.f * zz - 3.f) * c[63 + ch] +
                      SH_C4[6] * (xx - yy) * (7.f * zz - 1.f) * c[66 + ch] +
                      SH_C4[7] * xz * (xx - 3.f * yy) * c[69 + ch] +
                      SH_C4[8] * (xx * (xx - 3.f * yy) - yy * (3.f * xx - yy)) * c[72 + ch]);
            }
          }
        }
        rgbs[3 * (o + i) + ch] = fmaxf(acc + 0.5f, 0.f);
      }
    }
    project_point(i, px, py, pz, sc0, sc1, sc2, q0, q1, q2, q3, 1.f, vm, fx, fy, cx, cy, img_h, img_w, bw, 0.01f,
                  xys + 2 * o, depths + o, radii + o, conics + 3 * o, nullptr, num_tiles_hit + o, nullptr);
    if (rec) {  // the rasterizer's packed record (pack_raster_records_kernel's layout), from this thread's own stores
      const long long r = o + i;
      const float* xy = xys + 2 * r;
      const float* cn = conics + 3 * r;
      const float* cl = rgbs + 3 * r;
      rec[4 * r + 0] = make_float4(xy[0], xy[1], op, cn[0]);
      rec[4 * r + 1] = make_float4(cn[1], cn[2], cl[0], cl[1]);
      rec[4 * r + 2] = make_float4(cl[2], 0.f, 0.f, 0.f);
    }
  }
}

// launch over n Gaussians x nviews cameras (c2ws [nviews][4][4]; per-view outputs at view * n records)
int launch_prep(int n, int nviews, int num_bases, const float* means, const float* log_scales, const float* quats_raw,
                const float* opac_logit, const float* dc, const float* rest, PrepStrides ld, const float* c2ws,
                float fx, float fy, float cx, float cy, int img_h, int img_w, int bw, float* viewmat_out, float* rgbs,
                float* opac, float* xys, float* depths, int* radii, float* conics, int* num_tiles_hit,
                hipStream_t st, float* rec = nullptr) {
  const unsigned blocks = sfx::ceil_div(n > 0 ? n : 1, 256);
#define SFX_PREP(DG)                                                                                              \
  render_prep_project_kernel<DG><<<blocks, 256, 0, st>>>(n, nviews, means, log_scales, quats_raw, opac_logit, dc,  \
                                                         rest, ld, c2ws, fx, fy, cx, cy, img_h, img_w, bw,           \
                                                         viewmat_out, rgbs, opac, xys, depths, radii, conics,         \
                                                         num_tiles_hit, reinterpret_cast<float4*>(rec))
  switch (num_bases) {
    case 1: SFX_PREP(0); break;
    case 4: SFX_PREP(1); break;
    case 9: SFX_PREP(2); break;
    case 16: SFX_PREP(3); break;
    default: SFX_PREP(4); break;
  }
#undef SFX_PREP
  return SFX_OK;
}

// backward of project (gsplat project_gaussians_backward_kernel semantics: the
// EWA Jacobian uses the *unclamped* camera-space mean, and the quaternion
// gradient is taken w.r.t. the normalised quaternion).
__global__ void project_bwd_kernel(int n, const float* __restrict__ means, const float* __restrict__ scales,
                                   float glob_scale, const float* __restrict__ quats,
                                   const float* __restrict__ viewmat, float fx, float fy,
                                   const float* __restrict__ cov3d, const int* __restrict__ radii,
                                   const float* __restrict__ conics, const float* __restrict__ compensation,
                                   const float* __restrict__ v_xy, const float* __restrict__ v_depth,
                                   const float* __restrict__ v_conic, const float* __restrict__ v_comp,
                                   float* __restrict__ v_mean, float* __restrict__ v_scale,
                                   float* __restrict__ v_quat, float* __restrict__ v_cov2d,
                                   float* __restrict__ v_cov3d_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float vm_out[3] = {0.f, 0.f, 0.f}, vs_out[3] = {0.f, 0.f, 0.f}, vq_out[4] = {0.f, 0.f, 0.f, 0.f};
  float vc2[3] = {0.f, 0.f, 0.f}, vc3[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (radii[i] > 0) {
    float vm[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) vm[k] = viewmat[k];
    const float px = means[3 * i], py = means[3 * i + 1], pz = means[3 * i + 2];
    const float tx = vm[0] * px + vm[1] * py + vm[2] * pz + vm[3];
    const float ty = vm[4] * px + vm[5] * py + vm[6] * pz + vm[7];
    const float tz = vm[8] * px + vm[9] * py + vm[10] * pz + vm[11];
    // v_mean from v_xy (project_pix_vjp) + rot-only transpose
    {
      const float rw = 1.f / (tz + 1e-6f);
      const float vpx = fx * v_xy[2 * i], vpy = fy * v_xy[2 * i + 1];
      const float v0 = vpx * rw, v1 = vpy * rw, v2 = -(vpx * tx + vpy * ty) * rw * rw;
      vm_out[0] = vm[0] * v0 + vm[4] * v1 + vm[8] * v2;
      vm_out[1] = vm[1] * v0 + vm[5] * v1 + vm[9] * v2;
      vm_out[2] = vm[2] * v0 + vm[6] * v1 + vm[10] * v2;
      const float vz = v_depth[i];
      vm_out[0] += vm[8] * vz;
      vm_out[1] += vm[9] * vz;
      vm_out[2] += vm[10] * vz;
    }
    // v_cov2d from v_conic (cov2d_to_conic_vjp) and v_comp
    const float X0 = conics[3 * i], X1 = conics[3 * i + 1], X2 = conics[3 * i + 2];
    {
      const float G0 = v_conic[3 * i], G1 = 0.5f * v_conic[3 * i + 1], G2 = v_conic[3 * i + 2];
      // v_Sigma = -X G X  (symmetric 2x2)
      const float XG00 = X0 * G0 + X1 * G1, XG01 = X0 * G1 + X1 * G2;
      const float XG10 = X1 * G0 + X2 * G1, XG11 = X1 * G1 + X2 * G2;
      const float s00 = -(XG00 * X0 + XG01 * X1);
      const float s01 = -(XG00 * X1 + XG01 * X2);
      const float s10 = -(XG10 * X0 + XG11 * X1);
      const float s11 = -(XG10 * X1 + XG11 * X2);
      vc2[0] = s00;
      vc2[1] = s10 + s01;
      vc2[2] = s11;
      const float cmp = compensation[i];
      const float inv_det = X0 * X2 - X1 * X1;
      const float one_m = 1.f - cmp * cmp;
      const float vsq = v_comp[i] * 0.5f / (cmp + 1e-6f);
      vc2[0] += vsq * (one_m * X0 - 0.3f * inv_det);
      vc2[1] += 2.f * vsq * (one_m * X1);
      vc2[2] += vsq * (one_m * X2 - 0.3f * inv_det);
    }
    // v_cov3d and v_mean contribution (project_cov3d_ewa_vjp)
    const float* cv = cov3d + 6 * i;
    float V[3][3] = {{cv[0], cv[1], cv[2]}, {cv[1], cv[3], cv[4]}, {cv[2], cv[4], cv[5]}};
    const float rz = 1.f / tz, rz2 = rz * rz, rz3 = rz2 * rz;
    // T = J W (2 rows used; J row 2 is zero)
    const float j00 = fx * rz, j02 = -fx * tx * rz2, j11 = fy * rz, j12 = -fy * ty * rz2;
    float T[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      T[0][c] = j00 * vm[0 + c] + j02 * vm[8 + c];
      T[1][c] = j11 * vm[4 + c] + j12 * vm[8 + c];
      T[2][c] = 0.f;
    }
    float G[3][3] = {{vc2[0], 0.5f * vc2[1], 0.f}, {0.5f * vc2[1], vc2[2], 0.f}, {0.f, 0.f, 0.f}};
    // v_V = T^T G T
    float GT[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) GT[r][c] = G[r][0] * T[0][c] + G[r][1] * T[1][c] + G[r][2] * T[2][c];
    float vV[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) vV[r][c] = T[0][r] * GT[0][c] + T[1][r] * GT[1][c] + T[2][r] * GT[2][c];
    vc3[0] = vV[0][0];
    vc3[1] = vV[0][1] + vV[1][0];
    vc3[2] = vV[0][2] + vV[2][0];
    vc3[3] = vV[1][1];
    vc3[4] = vV[1][2] + vV[2][1];
    vc3[5] = vV[2][2];
    // v_T = G T V^T + G^T T V  (V symmetric, G symmetric -> 2 G T V)
    float vT[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float gtv = GT[r][0] * V[c][0] + GT[r][1] * V[c][1] + GT[r][2] * V[c][2];  // (G T V^T)[r][c]
        const float gtv2 = GT[r][0] * V[0][c] + GT[r][1] * V[1][c] + GT[r][2] * V[2][c];  // (G^T T V)[r][c]
        vT[r][c] = gtv + gtv2;
      }
    // v_J = v_T W^T
    float vJ[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) vJ[r][c] = vT[r][0] * vm[4 * c + 0] + vT[r][1] * vm[4 * c + 1] + vT[r][2] * vm[4 * c + 2];
    const float vt0 = -fx * rz2 * vJ[0][2];
    const float vt1 = -fy * rz2 * vJ[1][2];
    const float vt2 = -fx * rz2 * vJ[0][0] + 2.f * fx * tx * rz3 * vJ[0][2] - fy * rz2 * vJ[1][1] +
                      2.f * fy * ty * rz3 * vJ[1][2];
    vm_out[0] += vt0 * vm[0] + vt1 * vm[4] + vt2 * vm[8];
    vm_out[1] += vt0 * vm[1] + vt1 * vm[5] + vt2 * vm[9];
    vm_out[2] += vt0 * vm[2] + vt1 * vm[6] + vt2 * vm[10];

    // scale / quat (scale_rot_to_cov3d_vjp)
    const float qw = quats[4 * i], qx = quats[4 * i + 1], qy = quats[4 * i + 2], qz = quats[4 * i + 3];
    const M3 R = quat_to_rotmat(qw, qx, qy, qz);
    const float s[3] = {glob_scale * scales[3 * i], glob_scale * scales[3 * i + 1], glob_scale * scales[3 * i + 2]};
    float vVs[3][3] = {{vc3[0], 0.5f * vc3[1], 0.5f * vc3[2]},
                       {0.5f * vc3[1], vc3[3], 0.5f * vc3[4]},
                       {0.5f * vc3[2], 0.5f * vc3[4], vc3[5]}};
    float Mm[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) Mm[r][c] = R.m[r][c] * s[c];
    float vM[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) vM[r][c] = 2.f * (vVs[r][0] * Mm[0][c] + vVs[r][1] * Mm[1][c] + vVs[r][2] * Mm[2][c]);
#pragma unroll
    for (int c = 0; c < 3; ++c)
      vs_out[c] = (R.m[0][c] * vM[0][c] + R.m[1][c] * vM[1][c] + R.m[2][c] * vM[2][c]) * glob_scale;
    float vR[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) vR[r][c] = vM[r][c] * s[c];
    // quat_to_rotmat_vjp with glm column-major v_R[col][row] == vR[row][col]
    const float sn = rsqrtf(qw * qw + qx * qx + qy * qy + qz * qz);
    const float w = qw * sn, x = qx * sn, y = qy * sn, z = qz * sn;
#define VR(col, row) vR[row][col]
    vq_out[0] = 2.f * (x * (VR(1, 2) - VR(2, 1)) + y * (VR(2, 0) - VR(0, 2)) + z * (VR(0, 1) - VR(1, 0)));
    vq_out[1] = 2.f * (-2.f * x * (VR(1, 1) + VR(2, 2)) + y * (VR(0, 1) + VR(1, 0)) + z * (VR(0, 2) + VR(2, 0)) +
                       w * (VR(1, 2) - VR(2, 1)));
    vq_out[2] = 2.f * (x * (VR(0, 1) + VR(1, 0)) - 2.f * y * (VR(0, 0) + VR(2, 2)) + z * (VR(1, 2) + VR(2, 1)) +
                       w * (VR(2, 0) - VR(0, 2)));
    vq_out[3] = 2.f * (x * (VR(0, 2) + VR(2, 0)) + y * (VR(1, 2) + VR(2, 1)) - 2.f * z * (VR(0, 0) + VR(1, 1)) +
                       w * (VR(0, 1) - VR(1, 0)));
#undef VR
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    v_mean[3 * i + k] = vm_out[k];
    v_scale[3 * i + k] = vs_out[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) v_quat[4 * i + k] = vq_out[k];
  if (v_cov2d)
#pragma unroll
    for (int k = 0; k < 3; ++k) v_cov2d[3 * i + k] = vc2[k];
  if (v_cov3d_out)
#pragma unroll
    for (int k = 0; k < 6; ++k) v_cov3d_out[6 * i + k] = vc3[k];
}

// ---- intersections ----------------------------------------------------------
// n_per_view > 0: records are V views x n_per_view Gaussians; view v's tiles are numbered v*tiles_x*tiles_y + ...
__global__ void isect_emit_kernel(int n, const float* __restrict__ xys, const float* __restrict__ depths,
                                  const int* __restrict__ radii, const int* __restrict__ cum_tiles_hit,
                                  int tiles_x, int tiles_y, int bw, int64_t* __restrict__ isect_ids,
                                  int32_t* __restrict__ gaussian_ids, int n_per_view, int cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (radii[i] <= 0) return;
  int x0, y0, x1, y1;
  get_tile_bbox(xys[2 * i], xys[2 * i + 1], (float)radii[i], tiles_x, tiles_y, bw, x0, y0, x1, y1);
  // cap: the caller's buffer length -- a wrong prefix (a look-back scan that timed out) cannot write out of bounds
  int cur = (i == 0) ? 0 : max(cum_tiles_hit[i - 1], 0);
  const int64_t depth_id = (int64_t)__float_as_int(depths[i]);
  const int64_t tile_base = n_per_view > 0 ? (int64_t)(i / n_per_view) * tiles_x * tiles_y : 0;
  for (int ty = y0; ty < y1; ++ty)
    for (int tx = x0; tx < x1; ++tx) {
      if (cur >= cap) return;
      const int64_t tile_id = tile_base + (int64_t)ty * tiles_x + tx;
      isect_ids[cur] = (tile_id << 32) | (depth_id & 0xffffffffll);
      gaussian_ids[cur] = i;
      ++cur;
    }
}

__global__ void tile_bins_kernel(int num_isect, const int64_t* __restrict__ isect_sorted, int* __restrict__ tile_bins) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= num_isect) return;
  const int cur = (int)(isect_sorted[i] >> 32);
  if (i == 0) tile_bins[2 * cur] = 0;
  if (i == num_isect - 1) tile_bins[2 * cur + 1] = num_isect;
  if (i == 0) return;
  const int prev = (int)(isect_sorted[i - 1] >> 32);
  if (prev != cur) {
    tile_bins[2 * prev + 1] = i;
    tile_bins[2 * cur] = i;
  }
}

// ---- rasterize forward ------------------------------------------------------
constexpr int MAX_BLOCK = 256;

__global__ void __launch_bounds__(MAX_BLOCK)
rasterize_fwd_kernel(int tiles_x, int tiles_y, int bw, int img_h, int img_w,
                     const int32_t* __restrict__ gids_sorted, const int* __restrict__ tile_bins,
                     const float* __restrict__ xys, const float* __restrict__ conics,
                     const float* __restrict__ colors, const float* __restrict__ opacity,
                     const float* __restrict__ background, float* __restrict__ final_Ts,
                     int* __restrict__ final_idx, float* __restrict__ out_img, float* __restrict__ out_alpha,
                     int clamp_max1) {
  __shared__ int id_batch[MAX_BLOCK];
  __shared__ float4 xyo_batch[MAX_BLOCK];   // x, y, opacity, pad
  __shared__ float4 conic_batch[MAX_BLOCK]; // a, b, c, pad
  __shared__ float4 rgb_batch[MAX_BLOCK];

  // batched views: blockIdx.z = view (tiles numbered per view, per-view image planes)
  const int tile_id = blockIdx.z * tiles_x * tiles_y + blockIdx.y * tiles_x + blockIdx.x;
  if (blockIdx.z > 0) {
    const long long po = (long long)blockIdx.z * img_h * img_w;
    final_Ts += po; final_idx += po; out_img += 3 * po;
    if (out_alpha) out_alpha += po;
  }
  const int tr = threadIdx.x;  // flat thread rank, row-major over (ty, tx)
  const int ty = tr / bw, tx = tr - (tr / bw) * bw;
  const int block_size = bw * bw;
  const unsigned pi = blockIdx.y * bw + ty, pj = blockIdx.x * bw + tx;
  const float px = (float)pj + 0.5f, py = (float)pi + 0.5f;
  const bool inside = (pi < (unsigned)img_h && pj < (unsigned)img_w);
  bool done = !inside;

  const int range_x = tile_bins[2 * tile_id], range_y = tile_bins[2 * tile_id + 1];
  const int num_batches = (range_y - range_x + block_size - 1) / block_size;

  float T = 1.f;
  int cur_idx = 0;
  float r0 = 0.f, r1 = 0.f, r2 = 0.f;
  for (int b = 0; b < num_batches; ++b) {
    // resync before overwriting the batch; early exit when the whole tile is done
    if (__syncthreads_count(done) >= block_size) break;

    const int batch_start = range_x + block_size * b;
    const int idx = batch_start + tr;
    if (idx < range_y) {
      const int g = gids_sorted[idx];
      id_batch[tr] = g;
      xyo_batch[tr] = make_float4(xys[2 * g], xys[2 * g + 1], opacity[g], 0.f);
      conic_batch[tr] = make_float4(conics[3 * g], conics[3 * g + 1], conics[3 * g + 2], 0.f);
      rgb_batch[tr] = make_float4(colors[3 * g], colors[3 * g + 1], colors[3 * g + 2], 0.f);
    }
    __syncthreads();
    const int batch_size = min(block_size, range_y - batch_start);
    for (int t = 0; (t < batch_size) && !done; ++t) {
      const float4 con = conic_batch[t];
      const float4 xyo = xyo_batch[t];
      const float dx = xyo.x - px, dy = xyo.y - py;
      const float sigma = 0.5f * (con.x * dx * dx + con.z * dy * dy) + con.y * dx * dy;
      const float alpha = fminf(0.999f, xyo.z * __expf(-sigma));
      if (sigma < 0.f || alpha < 1.f / 255.f) continue;
      const float next_T = T * (1.f - alpha);
      if (next_T <= 1e-4f) {
        done = true;
        break;
      }
      const float vis = alpha * T;
      const float4 c = rgb_batch[t];
      r0 = r0 + c.x * vis;
      r1 = r1 + c.y * vis;
      r2 = r2 + c.z * vis;
      T = next_T;
      cur_idx = batch_start + t;
    }
  }
  if (inside) {
    const int pix = pi * img_w + pj;
    final_Ts[pix] = T;
    final_idx[pix] = cur_idx;
    float o0 = r0 + T * background[0], o1 = r1 + T * background[1], o2 = r2 + T * background[2];
    if (clamp_max1) {  // gs_utils.py:111 torch.clamp(rgb, max=1), fused for the eval path
      o0 = fminf(o0, 1.f); o1 = fminf(o1, 1.f); o2 = fminf(o2, 1.f);
    }
    out_img[3 * pix + 0] = o0;
    out_img[3 * pix + 1] = o1;
    out_img[3 * pix + 2] = o2;
    if (out_alpha) out_alpha[pix] = 1.f - T;
  }
}

// ---- packed records (eval path) ------------------------------------------------
// One 48-byte record per projected Gaussian, written once per view batch: r0 = (x, y, opacity, conic.a),
// r1 = (conic.b, conic.c, r, g), r2 = (b, 0, 0, 0), at a 64-byte stride (one 64-byte sector per record gather; at
// 48 bytes two of every four records straddle a sector boundary: 1.5 sectors fetched per 36 bytes used).  The rasterizer's per-batch fetch is one gather of a
// 16-byte-aligned record instead of four gathers from four arrays (xys 8 B, opacity 4 B, conics 12 B,
// colours 12 B).  Measured: the same kernel time as the four-array form (config E 2285 vs 2278 us for 9
// 1920x1080 views) -- the rasterizer is not bound by its gathers.  A wave-uniform skip of Gaussians whose
// alpha >= 1/255 ellipse misses the wave's 16 x 4 pixels (exact, extents in r2) was 25 % slower (2855 us) and
// is not kept.
__global__ void pack_raster_records_kernel(int n, const float* __restrict__ xys, const float* __restrict__ conics,
                                           const float* __restrict__ colors, const float* __restrict__ opacity,
                                           float4* __restrict__ rec) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  rec[4 * i + 0] = make_float4(xys[2 * i], xys[2 * i + 1], opacity[i], conics[3 * i]);
  rec[4 * i + 1] = make_float4(conics[3 * i + 1], conics[3 * i + 2], colors[3 * i], colors[3 * i + 1]);
  rec[4 * i + 2] = make_float4(colors[3 * i + 2], 0.f, 0.f, 0.f);
}

// rasterize_fwd_kernel over packed records: the same per-pixel arithmetic in the same order (bit-identical
// outputs); the batch is staged in LDS as the records themselves and r2 (blue) is read only for Gaussians
// that pass the alpha test.
__global__ void __launch_bounds__(MAX_BLOCK)
rasterize_fwd_packed_kernel(int tiles_x, int tiles_y, int bw, int img_h, int img_w,
                            const int32_t* __restrict__ gids_sorted, const int* __restrict__ tile_bins,
                            const float4* __restrict__ rec, const float* __restrict__ background,
                            float* __restrict__ final_Ts, int* __restrict__ final_idx, float* __restrict__ out_img,
                            float* __restrict__ out_alpha, int clamp_max1) {
  __shared__ float4 r0_batch[MAX_BLOCK];
  __shared__ float4 r1_batch[MAX_BLOCK];
  __shared__ float r2_batch[MAX_BLOCK];

  const int tile_id = blockIdx.z * tiles_x * tiles_y + blockIdx.y * tiles_x + blockIdx.x;
  if (blockIdx.z > 0) {
    const long long po = (long long)blockIdx.z * img_h * img_w;
    final_Ts += po; final_idx += po; out_img += 3 * po;
    if (out_alpha) out_alpha += po;
  }
  const int tr = threadIdx.x;
  const int ty = tr / bw, tx = tr - (tr / bw) * bw;
  const int block_size = bw * bw;
  const unsigned pi = blockIdx.y * bw + ty, pj = blockIdx.x * bw + tx;
  const float px = (float)pj + 0.5f, py = (float)pi + 0.5f;
  const bool inside = (pi < (unsigned)img_h && pj < (unsigned)img_w);
  bool done = !inside;

  const int range_x = tile_bins[2 * tile_id], range_y = tile_bins[2 * tile_id + 1];
  const int num_batches = (range_y - range_x + block_size - 1) / block_size;

  float T = 1.f;
  int cur_idx = 0;
  float c0 = 0.f, c1 = 0.f, c2 = 0.f;
  for (int b = 0; b < num_batches; ++b) {
    if (__syncthreads_count(done) >= block_size) break;
    const int batch_start = range_x + block_size * b;
    const int idx = batch_start + tr;
    if (idx < range_y) {
      const long long g = gids_sorted[idx];
      r0_batch[tr] = rec[4 * g];
      r1_batch[tr] = rec[4 * g + 1];
      r2_batch[tr] = reinterpret_cast<const float*>(rec + 4 * g + 2)[0];
    }
    __syncthreads();
    const int batch_size = min(block_size, range_y - batch_start);
    for (int t = 0; (t < batch_size) && !done; ++t) {
      const float4 a = r0_batch[t];
      const float4 q = r1_batch[t];
      const float dx = a.x - px, dy = a.y - py;
      const float sigma = 0.5f * (a.w * dx * dx + q.y * dy * dy) + q.x * dx * dy;
      const float alpha = fminf(0.999f, a.z * __expf(-sigma));
      if (sigma < 0.f || alpha < 1.f / 255.f) continue;
      const float next_T = T * (1.f - alpha);
      if (next_T <= 1e-4f) {
        done = true;
        break;
      }
      const float vis = alpha * T;
      c0 = c0 + q.z * vis;
      c1 = c1 + q.w * vis;
      c2 = c2 + r2_batch[t] * vis;
      T = next_T;
      cur_idx = batch_start + t;
    }
  }
  if (inside) {
    const int pix = pi * img_w + pj;
    final_Ts[pix] = T;
    final_idx[pix] = cur_idx;
    float o0 = c0 + T * background[0], o1 = c1 + T * background[1], o2 = c2 + T * background[2];
    if (clamp_max1) {
      o0 = fminf(o0, 1.f); o1 = fminf(o1, 1.f); o2 = fminf(o2, 1.f);
    }
    out_img[3 * pix + 0] = o0;
    out_img[3 * pix + 1] = o1;
    out_img[3 * pix + 2] = o2;
    if (out_alpha) out_alpha[pix] = 1.f - T;
  }
}

// ---- exact contribution culling (eval path, ABI v9) ---------------------------------------------------------
// gsplat bins a Gaussian into every tile of its 3-sigma square (get_tile_bbox) and the per-pixel loop then skips
// it wherever alpha = min(0.999, o exp(-sigma)) < 1/255.  A (Gaussian, pixel box) pair can be dropped without
// changing any output bit when no pixel centre in the box can pass that test: sigma is a positive-definite
// quadratic in d = (x, y) - pixel, so its minimum over the box of d is 0 (centre inside) or on an edge (a 1-D
// quadratic clamped to the edge).  The minimum is evaluated in fp32 and compared against a limit raised by
// margins far above every rounding involved: the kernel's own fp32 sigma (relative error <= a few ulp *
// (1 + rho) / (1 - rho), rho = |b| / sqrt(ac) <= 0.99 here), this evaluation, __expf / __logf (absolute 1e-4 on
// the log threshold).  Near-degenerate (rho > 0.99), non-PD and non-finite conics or positions are never
// dropped.  Dropped pairs are exactly ones the rasterizer would `continue` past for every pixel of the box, so
// images, alphas and final T are bit-identical; only final_idx (a list position) refers to the shorter list.
struct CullG {
  float gx, gy, a, b, c, ia, ic, lim;  // lim: box minimum of sigma above which the box is dropped
  bool never, always;                  // never: o < 1/255 everywhere; always: never drop (degenerate input)
};

__device__ __forceinline__ CullG cull_setup(float x, float y, float ca, float cb, float cc, float opac) {
  // no contraction here or in cull_box_may_hit: the count and emit kernels must take the same decision for every
  // (Gaussian, tile) (the emit walk fills exactly the slots the count reserved), whatever FMAs the compiler
  // would pick in each inlined copy
#pragma clang fp contract(off)
  CullG g;
  g.gx = x; g.gy = y; g.a = ca; g.b = cb; g.c = cc;
  g.ia = 0.f; g.ic = 0.f; g.lim = 0.f;
  g.always = false; g.never = false;
  const float ac = ca * cc;
  if (!(ca > 0.f) || !(cc > 0.f) || !(cb * cb < 0.9801f * ac) || !isfinite(x) || !isfinite(y) || !isfinite(ac)) {
    g.always = true;  // rho > 0.99, not positive definite, or non-finite
    return g;
  }
  if (!(opac * 255.f >= 0.999f)) {  // o < 1/255 (minus 1e-3): alpha < 1/255 at every pixel; NaN: keep
    if (opac * 255.f < 0.999f) g.never = true; else g.always = true;
    return g;
  }
  const float rho = sqrtf(cb * cb / ac);
  g.ia = 1.f / ca;
  g.ic = 1.f / cc;
  // may contribute iff sigma_min * (1 - 1e-4 / (1 - rho)) <= ln(255 o) + 2e-4
  g.lim = (__logf(opac * 255.f) + 2e-4f) / (1.f - 1e-4f / (1.f - rho));
  return g;
}

// May the Gaussian reach alpha >= 1/255 at a pixel centre of [px0, px1] x [py0, py1] (integer pixel bounds,
// inclusive, already clipped to the image)?
__device__ __forceinline__ bool cull_box_may_hit(const CullG& g, int px0, int px1, int py0, int py1) {
#pragma clang fp contract(off)
  if (g.always) return true;
  if (g.never || px0 > px1 || py0 > py1) return false;
  // d = g - (p + 0.5) over the pixel centres
  const float u0 = g.gx - ((float)px1 + 0.5f), u1 = g.gx - ((float)px0 + 0.5f);
  const float v0 = g.gy - ((float)py1 + 0.5f), v1 = g.gy - ((float)py0 + 0.5f);
  if (u0 <= 0.f && u1 >= 0.f && v0 <= 0.f && v1 >= 0.f) return true;
  float m = 3.0e38f;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float dx = e ? u1 : u0;
    const float dy = fminf(fmaxf(-g.b * dx * g.ic, v0), v1);
    m = fminf(m, 0.5f * (g.a * dx * dx + g.c * dy * dy) + g.b * dx * dy);
    const float ey = e ? v1 : v0;
    const float ex = fminf(fmaxf(-g.b * ey * g.ia, u0), u1);
    m = fminf(m, 0.5f * (g.a * ex * ex + g.c * ey * ey) + g.b * ex * ey);
  }
  return m <= g.lim;
}

// Tiles of a Gaussian's gsplat square are visited in gsplat's order (row-major over the square).  Squares of up
// to SMALL_AREA tiles are walked by their own lane; bigger ones (a few needles and near-camera Gaussians can
// cover thousands of tiles) by the whole wave, 64 tiles per step, so no lane serialises a long walk.
constexpr int CULL_SMALL_AREA = 16;

struct CullWalk {
  int x0, y0, x1, y1, area;
  CullG g;
};

__device__ __forceinline__ CullWalk cull_walk_setup(int i, const float* __restrict__ xys,
                                                    const float* __restrict__ conics, const float* __restrict__ opac,
                                                    const int* __restrict__ radii, int tiles_x, int tiles_y, int bw) {
  CullWalk w;
  w.x0 = w.y0 = w.x1 = w.y1 = 0;
  w.area = 0;
  if (radii[i] > 0) {
    get_tile_bbox(xys[2 * i], xys[2 * i + 1], (float)radii[i], tiles_x, tiles_y, bw, w.x0, w.y0, w.x1, w.y1);
    w.area = max(0, (w.x1 - w.x0) * (w.y1 - w.y0));
  }
  if (w.area > 0)
    w.g = cull_setup(xys[2 * i], xys[2 * i + 1], conics[3 * i], conics[3 * i + 1], conics[3 * i + 2], opac[i]);
  return w;
}

__device__ __forceinline__ CullG cull_bcast(const CullG& g, int l) {
  CullG o;
  o.gx = __shfl(g.gx, l); o.gy = __shfl(g.gy, l); o.a = __shfl(g.a, l); o.b = __shfl(g.b, l);
  o.c = __shfl(g.c, l); o.ia = __shfl(g.ia, l); o.ic = __shfl(g.ic, l); o.lim = __shfl(g.lim, l);
  o.never = __shfl((int)g.never, l) != 0;
  o.always = __shfl((int)g.always, l) != 0;
  return o;
}

// tiles of the gsplat 3-sigma square that survive the culling test.  256 threads, one Gaussian per lane.
__global__ void __launch_bounds__(256)
isect_count_cull_kernel(int n, int n_per_view, const float* __restrict__ xys, const float* __restrict__ conics,
                        const float* __restrict__ opac, const int* __restrict__ radii, int tiles_x, int tiles_y,
                        int bw, int img_h, int img_w, int* __restrict__ num_tiles_kept) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  CullWalk w;
  w.x0 = w.y0 = w.x1 = w.y1 = 0;  // empty walk for lanes without a Gaussian (or without surviving tiles)
  w.area = 0;
  w.g = cull_setup(0.f, 0.f, 0.f, 0.f, 0.f, 0.f);
  if (i < n) w = cull_walk_setup(i, xys, conics, opac, radii, tiles_x, tiles_y, bw);
  int cnt = 0;
  if (w.area <= CULL_SMALL_AREA) {
    for (int ty = w.y0; ty < w.y1; ++ty)
      for (int tx = w.x0; tx < w.x1; ++tx)
        cnt += cull_box_may_hit(w.g, tx * bw, min(tx * bw + bw, img_w) - 1, ty * bw, min(ty * bw + bw, img_h) - 1);
  }
  unsigned long long big = __ballot(w.area > CULL_SMALL_AREA);
  while (big) {
    const int l = __ffsll((long long)big) - 1;
    big &= big - 1;
    const CullG g = cull_bcast(w.g, l);
    const int x0 = __shfl(w.x0, l), y0 = __shfl(w.y0, l), wx = __shfl(w.x1, l) - x0, area = __shfl(w.area, l);
    int c = 0;
    for (int base = 0; base < area; base += 64) {
      const int k = base + lane;
      const int tx = x0 + k % wx, ty = y0 + k / wx;
      const bool hit = k < area &&
                       cull_box_may_hit(g, tx * bw, min(tx * bw + bw, img_w) - 1, ty * bw, min(ty * bw + bw, img_h) - 1);
      c += __popcll(__ballot(hit));
    }
    if (lane == l) cnt = c;
  }
  if (i < n) num_tiles_kept[i] = cnt;
}

// isect_emit_kernel over the surviving tiles only (same walk order: the list is a subsequence of gsplat's).
// rank (optional): Gaussian-view i is the rank[i]-th in emission order and cum_tiles_hit is over that order -- the
// depth order of the two-level sort (sfx_depth_keys), so the pairs only need a stable sort by tile.  Threads stay
// in index order (coalesced reads of the per-Gaussian inputs); only the output offsets follow the rank.
__global__ void __launch_bounds__(256)
isect_emit_cull_kernel(int n, int n_per_view, const float* __restrict__ xys, const float* __restrict__ conics,
                       const float* __restrict__ opac, const float* __restrict__ depths,
                       const int* __restrict__ radii, const int* __restrict__ cum_tiles_hit, int tiles_x,
                       int tiles_y, int bw, int img_h, int img_w, int64_t* __restrict__ isect_ids,
                       int32_t* __restrict__ gaussian_ids, const int* __restrict__ rank, int cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = (rank && i < n) ? rank[i] : i;
  const int lane = threadIdx.x & 63;
  CullWalk w;
  w.x0 = w.y0 = w.x1 = w.y1 = 0;  // empty walk for lanes without a Gaussian (or without surviving tiles)
  w.area = 0;
  w.g = cull_setup(0.f, 0.f, 0.f, 0.f, 0.f, 0.f);
  int cur = 0, end = 0;
  if (i < n) {
    // [cur, end) clamped into the caller's buffer [0, cap): a wrong prefix (a look-back scan that timed out, counted
    // by sfx_lookback_timeouts) yields a wrong list, never an out-of-bounds write
    cur = (j == 0) ? 0 : max(cum_tiles_hit[j - 1], 0);
    end = min(cum_tiles_hit[j], cap);
    if (end > cur) w = cull_walk_setup(i, xys, conics, opac, radii, tiles_x, tiles_y, bw);
  }
  const int64_t depth_id = i < n ? (int64_t)__float_as_int(depths[i]) & 0xffffffffll : 0;
  const int64_t tile_base = (int64_t)(i / n_per_view) * tiles_x * tiles_y;
  if (w.area <= CULL_SMALL_AREA) {
    for (int ty = w.y0; ty < w.y1; ++ty)
      for (int tx = w.x0; tx < w.x1; ++tx) {
        if (!cull_box_may_hit(w.g, tx * bw, min(tx * bw + bw, img_w) - 1, ty * bw, min(ty * bw + bw, img_h) - 1))
          continue;
        if (cur >= end) break;  // never taken: the count kernel ran the same test on the same inputs
        isect_ids[cur] = ((tile_base + (int64_t)ty * tiles_x + tx) << 32) | depth_id;
        gaussian_ids[cur] = i;
        ++cur;
      }
  }
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  unsigned long long big = __ballot(w.area > CULL_SMALL_AREA);
  while (big) {
    const int l = __ffsll((long long)big) - 1;
    big &= big - 1;
    const CullG g = cull_bcast(w.g, l);
    const int x0 = __shfl(w.x0, l), y0 = __shfl(w.y0, l), wx = __shfl(w.x1, l) - x0, area = __shfl(w.area, l);
    int pos = __shfl(cur, l);
    const int stop = __shfl(end, l);
    const int gi = __shfl(i, l);
    const int64_t d = (int64_t)__shfl((long long)depth_id, l);
    const int64_t tb = (int64_t)__shfl((long long)tile_base, l);
    for (int base = 0; base < area; base += 64) {
      const int k = base + lane;
      const int tx = x0 + k % wx, ty = y0 + k / wx;
      const bool hit = k < area &&
                       cull_box_may_hit(g, tx * bw, min(tx * bw + bw, img_w) - 1, ty * bw, min(ty * bw + bw, img_h) - 1);
      const unsigned long long bal = __ballot(hit);
      const int p = pos + __popcll(bal & lt_mask);
      if (hit && p < stop) {
        isect_ids[p] = ((tb + (int64_t)ty * tiles_x + tx) << 32) | d;
        gaussian_ids[p] = gi;
      }
      pos += __popcll(bal);
    }
  }
}

// inv[perm[j]] = j
__global__ void __launch_bounds__(256) invert_perm_kernel(long long n, const int* __restrict__ perm,
                                                          int* __restrict__ inv) {
  const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
  if (j < n) inv[perm[j]] = (int)j;
}

// keys[i] = the bit pattern of depths[i] (u64, upper half 0): the depth half of gsplat's (tile << 32 | depth) key
__global__ void __launch_bounds__(256) depth_keys_kernel(long long n, const float* __restrict__ depths,
                                                         uint64_t* __restrict__ keys) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) keys[i] = (uint64_t)(unsigned)__float_as_int(depths[i]);
}

// rasterize_fwd_packed_kernel with per-wave Gaussian lists: the 16x16 tile is split into four 8x8 quadrants, one
// per wave; while a batch is staged each lane tests its record against the four quadrants (cull_box_may_hit)
// and every wave compacts the batch to the records that can reach its quadrant.  Each pixel still visits its
// tile's Gaussians in list order and runs the identical arithmetic; it only skips records whose alpha is below
// 1/255 at all of its quadrant's pixel centres -- the ones the per-pixel test would `continue` past -- so every
// output is bit-identical to rasterize_fwd_packed_kernel over the same list.  bw must be 16.
__global__ void __launch_bounds__(MAX_BLOCK)
rasterize_fwd_quad_kernel(int tiles_x, int tiles_y, int img_h, int img_w, const int32_t* __restrict__ gids_sorted,
                          const int* __restrict__ tile_bins, const float4* __restrict__ rec,
                          const float* __restrict__ background, float* __restrict__ final_Ts,
                          int* __restrict__ final_idx, float* __restrict__ out_img, float* __restrict__ out_alpha,
                          int clamp_max1) {
  // the per-pixel arithmetic spelled out with the exact contractions the compiler gives
  // rasterize_fwd_packed_kernel / rasterize_fwd_kernel (their ISA: sigma = fma(dy, qx dx, 0.5 fma(dx, aw dx,
  // dy (qy dy))), colour += vis c as fma, out = fma(T, bg, colour)), so the outputs match them bit for bit
#pragma clang fp contract(off)
  constexpr int BW = 16, BS = BW * BW;
  __shared__ float4 r0_batch[BS];
  __shared__ float4 r1_batch[BS];
  __shared__ float r2_batch[BS];
  __shared__ unsigned char mask_batch[BS];
  __shared__ unsigned char wlist[4][BS];

  const int tile_id = blockIdx.z * tiles_x * tiles_y + blockIdx.y * tiles_x + blockIdx.x;
  if (blockIdx.z > 0) {
    const long long po = (long long)blockIdx.z * img_h * img_w;
    final_Ts += po; final_idx += po; out_img += 3 * po;
    if (out_alpha) out_alpha += po;
  }
  const int tr = threadIdx.x;
  const int lane = tr & 63, w = tr >> 6;
  const int qx = (w & 1) * 8, qy = (w >> 1) * 8;
  const unsigned pi = blockIdx.y * BW + qy + (lane >> 3), pj = blockIdx.x * BW + qx + (lane & 7);
  const float px = (float)pj + 0.5f, py = (float)pi + 0.5f;
  const bool inside = (pi < (unsigned)img_h && pj < (unsigned)img_w);
  bool done = !inside;
  // quadrant pixel boxes (clipped to the image) for the mask test
  const int tx0 = blockIdx.x * BW, ty0 = blockIdx.y * BW;

  const int range_x = tile_bins[2 * tile_id], range_y = tile_bins[2 * tile_id + 1];
  const int num_batches = (range_y - range_x + BS - 1) / BS;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  float T = 1.f;
  int cur_idx = 0;
  float c0 = 0.f, c1 = 0.f, c2 = 0.f;
  for (int b = 0; b < num_batches; ++b) {
    if (__syncthreads_count(done) >= BS) break;
    const int batch_start = range_x + BS * b;
    const int idx = batch_start + tr;
    unsigned m = 0;
    if (idx < range_y) {
      const long long g = gids_sorted[idx];
      const float4 a = rec[4 * g];
      const float4 q = rec[4 * g + 1];
      r0_batch[tr] = a;
      r1_batch[tr] = q;
      r2_batch[tr] = reinterpret_cast<const float*>(rec + 4 * g + 2)[0];
      const CullG cg = cull_setup(a.x, a.y, a.w, q.x, q.y, a.z);
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int bx0 = tx0 + (qd & 1) * 8, by0 = ty0 + (qd >> 1) * 8;
        m |= (unsigned)cull_box_may_hit(cg, bx0, min(bx0 + 8, img_w) - 1, by0, min(by0 + 8, img_h) - 1) << qd;
      }
    }
    mask_batch[tr] = (unsigned char)m;
    __syncthreads();
    // this wave's list: batch positions whose record may reach the quadrant, in batch order
    int cnt = 0;
#pragma unroll
    for (int ch = 0; ch < BS / 64; ++ch) {
      const bool hit = (mask_batch[ch * 64 + lane] >> w) & 1;
      const unsigned long long bal = __ballot(hit);
      if (hit) wlist[w][cnt + __popcll(bal & lt_mask)] = (unsigned char)(ch * 64 + lane);
      cnt += __popcll(bal);
    }
    __syncthreads();
    for (int j = 0; (j < cnt) && !done; ++j) {
      const int t = wlist[w][j];
      const float4 a = r0_batch[t];
      const float4 q = r1_batch[t];
      const float dx = a.x - px, dy = a.y - py;
      const float sigma = __builtin_fmaf(dy, q.x * dx, 0.5f * __builtin_fmaf(dx, a.w * dx, dy * (q.y * dy)));
      const float alpha = fminf(0.999f, a.z * __expf(-sigma));
      if (sigma < 0.f || alpha < 1.f / 255.f) continue;
      const float next_T = T * (1.f - alpha);
      if (next_T <= 1e-4f) {
        done = true;
        break;
      }
      const float vis = alpha * T;
      c0 = __builtin_fmaf(vis, q.z, c0);
      c1 = __builtin_fmaf(vis, q.w, c1);
      c2 = __builtin_fmaf(vis, r2_batch[t], c2);
      T = next_T;
      cur_idx = batch_start + t;
    }
  }
  if (inside) {
    const int pix = pi * img_w + pj;
    final_Ts[pix] = T;
    final_idx[pix] = cur_idx;
    float o0 = __builtin_fmaf(T, background[0], c0), o1 = __builtin_fmaf(T, background[1], c1),
          o2 = __builtin_fmaf(T, background[2], c2);
    if (clamp_max1) {
      o0 = fminf(o0, 1.f); o1 = fminf(o1, 1.f); o2 = fminf(o2, 1.f);
    }
    out_img[3 * pix + 0] = o0;
    out_img[3 * pix + 1] = o1;
    out_img[3 * pix + 2] = o2;
    if (out_alpha) out_alpha[pix] = 1.f - T;
  }
}

// ---- rasterize backward -----------------------------------------------------
__global__ void __launch_bounds__(MAX_BLOCK)
rasterize_bwd_kernel(int tiles_x, int tiles_y, int bw, int img_h, int img_w,
                     const int32_t* __restrict__ gids_sorted, const int* __restrict__ tile_bins,
                     const float* __restrict__ xys, const float* __restrict__ conics,
                     const float* __restrict__ colors, const float* __restrict__ opacity,
                     const float* __restrict__ background, const float* __restrict__ final_Ts,
                     const int* __restrict__ final_idx, const float* __restrict__ v_out,
                     const float* __restrict__ v_out_alpha, float* __restrict__ v_xy,
                     float* __restrict__ v_xy_abs, float* __restrict__ v_conic, float* __restrict__ v_rgb,
                     float* __restrict__ v_opacity) {
  __shared__ int id_batch[MAX_BLOCK];
  __shared__ float4 xyo_batch[MAX_BLOCK];
  __shared__ float4 conic_batch[MAX_BLOCK];
  __shared__ float4 rgb_batch[MAX_BLOCK];

  const int tile_id = blockIdx.y * tiles_x + blockIdx.x;
  const int tr = threadIdx.x;
  const int ty = tr / bw, tx = tr - (tr / bw) * bw;
  const int block_size = bw * bw;
  const unsigned pi = blockIdx.y * bw + ty, pj = blockIdx.x * bw + tx;
  const float px = (float)pj + 0.5f, py = (float)pi + 0.5f;
  const bool inside = (pi < (unsigned)img_h && pj < (unsigned)img_w);
  const int pix = min((int)(pi * img_w + pj), img_w * img_h - 1);

  const float T_final = final_Ts[pix];
  float T = T_final;
  float buf0 = 0.f, buf1 = 0.f, buf2 = 0.f;
  const int bin_final = inside ? final_idx[pix] : 0;
  const int range_x = tile_bins[2 * tile_id], range_y = tile_bins[2 * tile_id + 1];
  const int num_batches = (range_y - range_x + block_size - 1) / block_size;
  const float vo0 = v_out[3 * pix], vo1 = v_out[3 * pix + 1], vo2 = v_out[3 * pix + 2];
  const float voa = v_out_alpha ? v_out_alpha[pix] : 0.f;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  const int wave_bin_final = sfx::wave_max_i(bin_final);
  const int lane = threadIdx.x & 63;

  for (int b = 0; b < num_batches; ++b) {
    __syncthreads();
    const int batch_end = range_y - 1 - block_size * b;
    const int batch_size = min(block_size, batch_end + 1 - range_x);
    const int idx = batch_end - tr;
    if (idx >= range_x) {
      const int g = gids_sorted[idx];
      id_batch[tr] = g;
      xyo_batch[tr] = make_float4(xys[2 * g], xys[2 * g + 1], opacity[g], 0.f);
      conic_batch[tr] = make_float4(conics[3 * g], conics[3 * g + 1], conics[3 * g + 2], 0.f);
      rgb_batch[tr] = make_float4(colors[3 * g], colors[3 * g + 1], colors[3 * g + 2], 0.f);
    }
    __syncthreads();
    for (int t = max(0, batch_end - wave_bin_final); t < batch_size; ++t) {
      bool valid = inside && (batch_end - t <= bin_final);
      float alpha = 0.f, opac = 0.f, vis = 0.f, dx = 0.f, dy = 0.f;
      float4 con = make_float4(0.f, 0.f, 0.f, 0.f);
      if (valid) {
        con = conic_batch[t];
        const float4 xyo = xyo_batch[t];
        opac = xyo.z;
        dx = xyo.x - px;
        dy = xyo.y - py;
        const float sigma = 0.5f * (con.x * dx * dx + con.z * dy * dy) + con.y * dx * dy;
        vis = __expf(-sigma);
        alpha = fminf(0.99f, opac * vis);
        if (sigma < 0.f || alpha < 1.f / 255.f) valid = false;
      }
      if (!__any(valid)) continue;
      float g_rgb0 = 0.f, g_rgb1 = 0.f, g_rgb2 = 0.f, g_c0 = 0.f, g_c1 = 0.f, g_c2 = 0.f;
      float g_xy0 = 0.f, g_xy1 = 0.f, g_ax = 0.f, g_ay = 0.f, g_o = 0.f;
      if (valid) {
        const float ra = 1.f / (1.f - alpha);
        T *= ra;
        const float fac = alpha * T;
        g_rgb0 = fac * vo0;
        g_rgb1 = fac * vo1;
        g_rgb2 = fac * vo2;
        const float4 rgb = rgb_batch[t];
        float v_alpha = 0.f;
        v_alpha += (rgb.x * T - buf0 * ra) * vo0;
        v_alpha += (rgb.y * T - buf1 * ra) * vo1;
        v_alpha += (rgb.z * T - buf2 * ra) * vo2;
        v_alpha += T_final * ra * voa;
        v_alpha += -T_final * ra * bg0 * vo0;
        v_alpha += -T_final * ra * bg1 * vo1;
        v_alpha += -T_final * ra * bg2 * vo2;
        buf0 += rgb.x * fac;
        buf1 += rgb.y * fac;
        buf2 += rgb.z * fac;
        const float v_sigma = -opac * vis * v_alpha;
        g_c0 = 0.5f * v_sigma * dx * dx;
        g_c1 = v_sigma * dx * dy;
        g_c2 = 0.5f * v_sigma * dy * dy;
        g_xy0 = v_sigma * (con.x * dx + con.y * dy);
        g_xy1 = v_sigma * (con.y * dx + con.z * dy);
        g_ax = fabsf(g_xy0);
        g_ay = fabsf(g_xy1);
        g_o = vis * v_alpha;
      }
      g_rgb0 = sfx::wave_sum_dpp(g_rgb0);
      g_rgb1 = sfx::wave_sum_dpp(g_rgb1);
      g_rgb2 = sfx::wave_sum_dpp(g_rgb2);
      g_c0 = sfx::wave_sum_dpp(g_c0);
      g_c1 = sfx::wave_sum_dpp(g_c1);
      g_c2 = sfx::wave_sum_dpp(g_c2);
      g_xy0 = sfx::wave_sum_dpp(g_xy0);
      g_xy1 = sfx::wave_sum_dpp(g_xy1);
      g_o = sfx::wave_sum_dpp(g_o);
      if (v_xy_abs) {
        g_ax = sfx::wave_sum_dpp(g_ax);
        g_ay = sfx::wave_sum_dpp(g_ay);
      }
      if (lane == 0) {
        const int g = id_batch[t];
        atomicAdd(v_rgb + 3 * g + 0, g_rgb0);
        atomicAdd(v_rgb + 3 * g + 1, g_rgb1);
        atomicAdd(v_rgb + 3 * g + 2, g_rgb2);
        atomicAdd(v_conic + 3 * g + 0, g_c0);
        atomicAdd(v_conic + 3 * g + 1, g_c1);
        atomicAdd(v_conic + 3 * g + 2, g_c2);
        atomicAdd(v_xy + 2 * g + 0, g_xy0);
        atomicAdd(v_xy + 2 * g + 1, g_xy1);
        if (v_xy_abs) {
          atomicAdd(v_xy_abs + 2 * g + 0, g_ax);
          atomicAdd(v_xy_abs + 2 * g + 1, g_ay);
        }
        atomicAdd(v_opacity + g, g_o);
      }
    }
  }
}

// rasterize_bwd_kernel over a culled list with rasterize_fwd_quad_kernel's layout: one 8x8 quadrant per wave
// and, per batch, per-wave lists of the records that can reach the quadrant (cull_box_may_hit) and lie at or
// before the wave's last contributing position (final_idx).  Every skipped record has alpha < 1/255 at each
// pixel of the quadrant -- the per-pixel `valid` test would be false for all lanes -- so each pixel sees the same
// contributions in the same back-to-front order; per-Gaussian sums per wave as before (one atomic per wave and
// Gaussian that any lane of the wave touches).  bw = 16.
__global__ void __launch_bounds__(MAX_BLOCK)
rasterize_bwd_quad_kernel(int tiles_x, int tiles_y, int img_h, int img_w, const int32_t* __restrict__ gids_sorted,
                          const int* __restrict__ tile_bins, const float* __restrict__ xys,
                          const float* __restrict__ conics, const float* __restrict__ colors,
                          const float* __restrict__ opacity, const float* __restrict__ background,
                          const float* __restrict__ final_Ts, const int* __restrict__ final_idx,
                          const float* __restrict__ v_out, const float* __restrict__ v_out_alpha,
                          float* __restrict__ v_xy, float* __restrict__ v_xy_abs, float* __restrict__ v_conic,
                          float* __restrict__ v_rgb, float* __restrict__ v_opacity) {
  constexpr int BW = 16, BS = BW * BW;
  __shared__ int id_batch[BS];
  __shared__ float4 xyo_batch[BS];
  __shared__ float4 conic_batch[BS];
  __shared__ float4 rgb_batch[BS];
  __shared__ unsigned char mask_batch[BS];
  __shared__ unsigned char wlist[4][BS];

  const int tile_id = blockIdx.y * tiles_x + blockIdx.x;
  const int tr = threadIdx.x;
  const int lane = tr & 63, w = tr >> 6;
  const int qx = (w & 1) * 8, qy = (w >> 1) * 8;
  const unsigned pi = blockIdx.y * BW + qy + (lane >> 3), pj = blockIdx.x * BW + qx + (lane & 7);
  const float px = (float)pj + 0.5f, py = (float)pi + 0.5f;
  const bool inside = (pi < (unsigned)img_h && pj < (unsigned)img_w);
  const int pix = min((int)(pi * img_w + pj), img_w * img_h - 1);
  const int tx0 = blockIdx.x * BW, ty0 = blockIdx.y * BW;

  const float T_final = final_Ts[pix];
  float T = T_final;
  float buf0 = 0.f, buf1 = 0.f, buf2 = 0.f;
  const int bin_final = inside ? final_idx[pix] : 0;
  const int range_x = tile_bins[2 * tile_id], range_y = tile_bins[2 * tile_id + 1];
  const int num_batches = (range_y - range_x + BS - 1) / BS;
  const float vo0 = v_out[3 * pix], vo1 = v_out[3 * pix + 1], vo2 = v_out[3 * pix + 2];
  const float voa = v_out_alpha ? v_out_alpha[pix] : 0.f;
  const float bg0 = background[0], bg1 = background[1], bg2 = background[2];
  const int wave_bin_final = sfx::wave_max_i(inside ? bin_final : -1);
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  constexpr int RING = 8;
  __shared__ float ring[4][RING][12][4];
  __shared__ int ring_g[4][RING];
  int nring = 0;  // records parked in this wave's ring (wave-uniform)
  auto flush_ring = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nv = v_xy_abs ? 11 : 9;
    for (int e = lane; e < nring * nv; e += 64) {
      const int jj = e / nv, c = e - jj * nv;
      const float* q = ring[w][jj][c];
      const float sum = (q[0] + q[1]) + (q[2] + q[3]);
      const int g = ring_g[w][jj];
      float* dst = c < 3 ? v_rgb + 3 * g + c
                 : c < 6 ? v_conic + 3 * g + (c - 3)
                 : c < 8 ? v_xy + 2 * g + (c - 6)
                 : c == 8 ? v_opacity + g
                          : v_xy_abs + 2 * g + (c - 9);
      atomicAdd(dst, sum);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    nring = 0;
  };

  for (int b = 0; b < num_batches; ++b) {
    __syncthreads();
    const int batch_end = range_y - 1 - BS * b;
    const int idx = batch_end - tr;
    unsigned m = 0;
    if (idx >= range_x) {
      const int g = gids_sorted[idx];
      const float4 xyo = make_float4(xys[2 * g], xys[2 * g + 1], opacity[g], 0.f);
      const float4 con = make_float4(conics[3 * g], conics[3 * g + 1], conics[3 * g + 2], 0.f);
      id_batch[tr] = g;
      xyo_batch[tr] = xyo;
      conic_batch[tr] = con;
      rgb_batch[tr] = make_float4(colors[3 * g], colors[3 * g + 1], colors[3 * g + 2], 0.f);
      const CullG cg = cull_setup(xyo.x, xyo.y, con.x, con.y, con.z, xyo.z);
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int bx0 = tx0 + (qd & 1) * 8, by0 = ty0 + (qd >> 1) * 8;
        m |= (unsigned)cull_box_may_hit(cg, bx0, min(bx0 + 8, img_w) - 1, by0, min(by0 + 8, img_h) - 1) << qd;
      }
    }
    mask_batch[tr] = (unsigned char)m;
    __syncthreads();
    int cnt = 0;
#pragma unroll
    for (int ch = 0; ch < BS / 64; ++ch) {
      const int t = ch * 64 + lane;
      const bool hit = ((mask_batch[t] >> w) & 1) && (batch_end - t <= wave_bin_final);
      const unsigned long long bal = __ballot(hit);
      if (hit) wlist[w][cnt + __popcll(bal & lt_mask)] = (unsigned char)t;
      cnt += __popcll(bal);
    }
    __syncthreads();
    for (int j = 0; j < cnt; ++j) {
      const int t = wlist[w][j];
      bool valid = inside && (batch_end - t <= bin_final);
      float alpha = 0.f, opac = 0.f, vis = 0.f, dx = 0.f, dy = 0.f;
      float4 con = make_float4(0.f, 0.f, 0.f, 0.f);
      if (valid) {
        con = conic_batch[t];
        const float4 xyo = xyo_batch[t];
        opac = xyo.z;
        dx = xyo.x - px;
        dy = xyo.y - py;
        const float sigma = 0.5f * (con.x * dx * dx + con.z * dy * dy) + con.y * dx * dy;
        vis = __expf(-sigma);
        alpha = fminf(0.99f, opac * vis);
        if (sigma < 0.f || alpha < 1.f / 255.f) valid = false;
      }
      if (!__any(valid)) continue;
      float g_rgb0 = 0.f, g_rgb1 = 0.f, g_rgb2 = 0.f, g_c0 = 0.f, g_c1 = 0.f, g_c2 = 0.f;
      float g_xy0 = 0.f, g_xy1 = 0.f, g_ax = 0.f, g_ay = 0.f, g_o = 0.f;
      if (valid) {
        const float ra = 1.f / (1.f - alpha);
        T *= ra;
        const float fac = alpha * T;
        g_rgb0 = fac * vo0;
        g_rgb1 = fac * vo1;
        g_rgb2 = fac * vo2;
        const float4 rgb = rgb_batch[t];
        float v_alpha = 0.f;
        v_alpha += (rgb.x * T - buf0 * ra) * vo0;
        v_alpha += (rgb.y * T - buf1 * ra) * vo1;
        v_alpha += (rgb.z * T - buf2 * ra) * vo2;
        v_alpha += T_final * ra * voa;
        v_alpha += -T_final * ra * bg0 * vo0;
        v_alpha += -T_final * ra * bg1 * vo1;
        v_alpha += -T_final * ra * bg2 * vo2;
        buf0 += rgb.x * fac;
        buf1 += rgb.y * fac;
        buf2 += rgb.z * fac;
        const float v_sigma = -opac * vis * v_alpha;
        g_c0 = 0.5f * v_sigma * dx * dx;
        g_c1 = v_sigma * dx * dy;
        g_c2 = 0.5f * v_sigma * dy * dy;
        g_xy0 = v_sigma * (con.x * dx + con.y * dy);
        g_xy1 = v_sigma * (con.y * dx + con.z * dy);
        g_ax = fabsf(g_xy0);
        g_ay = fabsf(g_xy1);
        g_o = vis * v_alpha;
      }
      // row sums of the 12 slots by a transposing butterfly: lane bit 0 then bit 1 split the slots between the
      // two partners (each keeps half, adds the other's copy of it: 12 -> 6 -> 3 slots per lane), then two
      // rotations sum the row's 4 quads -- 6 + 3 + 6 DPP moves instead of 4 per slot.  Lane (l & 3) of each row
      // then holds slots 6 (l & 1) + 3 ((l >> 1) & 1) + {0, 1, 2}, parked in this wave's LDS ring; the 4 row
      // partials of 8 records are added and sent with one atomic per (record, value) by the wave's lanes in
      // parallel (flush below)
      const float vals[12] = {g_rgb0, g_rgb1, g_rgb2, g_c0, g_c1, g_c2, g_xy0, g_xy1, g_o, g_ax, g_ay, 0.f};
      const bool hi0 = lane & 1, hi1 = lane & 2;
      float h6[6], h3[3];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float keep = hi0 ? vals[i + 6] : vals[i], send = hi0 ? vals[i] : vals[i + 6];
        h6[i] = keep + sfx::dpp_mov<0xB1>(send);  // quad [1,0,3,2]
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float keep = hi1 ? h6[i + 3] : h6[i], send = hi1 ? h6[i] : h6[i + 3];
        h3[i] = keep + sfx::dpp_mov<0x4E>(send);  // quad [2,3,0,1]
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) h3[i] += sfx::dpp_mov<0x124>(h3[i]);  // row_ror:4
#pragma unroll
      for (int i = 0; i < 3; ++i) h3[i] += sfx::dpp_mov<0x128>(h3[i]);  // row_ror:8
      if ((lane & 15) < 4) {
        const int base = 6 * (lane & 1) + 3 * ((lane >> 1) & 1);
#pragma unroll
        for (int i = 0; i < 3; ++i) ring[w][nring][base + i][lane >> 4] = h3[i];
      }
      if (lane == 0) ring_g[w][nring] = id_batch[t];
      if (++nring == RING) flush_ring();
    }
  }
  flush_ring();
}

}  // namespace

extern "C" {

int sfx_sh_fwd(int n, int num_bases, int degrees_to_use, const float* viewdirs, const float* coeffs, float* colors,
               void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_sh_fwd: n < 0");
  SFX_REQUIRE(degrees_to_use >= 0 && degrees_to_use <= 4, "sfx_sh_fwd: degrees_to_use must be in [0,4]");
  SFX_REQUIRE((degrees_to_use + 1) * (degrees_to_use + 1) <= num_bases, "sfx_sh_fwd: coeffs has too few bases");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(viewdirs && coeffs && colors, "sfx_sh_fwd: null buffer");
  sh_fwd_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, num_bases, degrees_to_use, viewdirs,
                                                                            coeffs, colors);
  return sfx::check_launch("sfx_sh_fwd");
}

int sfx_sh_bwd(int n, int num_bases, int degrees_to_use, const float* viewdirs, const float* v_colors,
               float* v_coeffs, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_sh_bwd: n < 0");
  SFX_REQUIRE(degrees_to_use >= 0 && degrees_to_use <= 4, "sfx_sh_bwd: degrees_to_use must be in [0,4]");
  SFX_REQUIRE((degrees_to_use + 1) * (degrees_to_use + 1) <= num_bases, "sfx_sh_bwd: coeffs has too few bases");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(viewdirs && v_colors && v_coeffs, "sfx_sh_bwd: null buffer");
  sh_bwd_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, num_bases, degrees_to_use, viewdirs,
                                                                            v_colors, v_coeffs);
  return sfx::check_launch("sfx_sh_bwd");
}

int sfx_project_fwd(int n, const float* means, const float* scales, float glob_scale, const float* quats,
                    const float* viewmat, float fx, float fy, float cx, float cy, int img_h, int img_w,
                    int block_width, float clip_thresh, float* xys, float* depths, int* radii, float* conics,
                    float* compensation, int* num_tiles_hit, float* cov3d, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_project_fwd: n < 0");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_project_fwd: block_width must be in (1,16]");
  SFX_REQUIRE(img_h > 0 && img_w > 0, "sfx_project_fwd: empty image");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(means && scales && quats && viewmat && xys && depths && radii && conics && compensation &&
                  num_tiles_hit && cov3d,
              "sfx_project_fwd: null buffer");
  project_fwd_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(
      n, means, scales, glob_scale, quats, viewmat, fx, fy, cx, cy, img_h, img_w, block_width, clip_thresh, xys,
      depths, radii, conics, compensation, num_tiles_hit, cov3d);
  return sfx::check_launch("sfx_project_fwd");
}

int sfx_render_prep_project(int n, int num_bases, const float* means, long long ld_means, const float* log_scales,
                            long long ld_scales, const float* quats_raw, long long ld_quats, const float* opac_logit,
                            long long ld_opac, const float* features_dc, long long ld_dc, const float* features_rest,
                            long long ld_rest, const float* camera_to_world, float fx, float fy, float cx,
                            float cy, int img_h, int img_w, int block_width, float* viewmat_out, float* rgbs,
                            float* opacities, float* xys, float* depths, int* radii, float* conics,
                            int* num_tiles_hit, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_render_prep_project: n < 0");
  SFX_REQUIRE(num_bases == 1 || num_bases == 4 || num_bases == 9 || num_bases == 16 || num_bases == 25,
              "sfx_render_prep_project: num_bases must be a square in {1,4,9,16,25}");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_render_prep_project: block_width must be in (1,16]");
  SFX_REQUIRE(img_h > 0 && img_w > 0, "sfx_render_prep_project: empty image");
  SFX_REQUIRE(camera_to_world, "sfx_render_prep_project: null camera");
  if (n > 0)
    SFX_REQUIRE(means && log_scales && quats_raw && opac_logit && features_dc && (num_bases == 1 || features_rest) &&
                    rgbs && opacities && xys && depths && radii && conics && num_tiles_hit,
                "sfx_render_prep_project: null buffer");
  launch_prep(n, 1, num_bases, means, log_scales, quats_raw, opac_logit, features_dc, features_rest,
              PrepStrides{ld_means, ld_scales, ld_quats, ld_opac, ld_dc, ld_rest}, camera_to_world, fx, fy, cx, cy,
              img_h, img_w, block_width, viewmat_out, rgbs, opacities, xys, depths, radii, conics, num_tiles_hit,
              sfx::as_stream(stream));
  return sfx::check_launch("sfx_render_prep_project");
}

int sfx_project_bwd(int n, const float* means, const float* scales, float glob_scale, const float* quats,
                    const float* viewmat, float fx, float fy, const float* cov3d, const int* radii,
                    const float* conics, const float* compensation, const float* v_xy, const float* v_depth,
                    const float* v_conic, const float* v_compensation, float* v_mean, float* v_scale,
                    float* v_quat, float* v_cov2d, float* v_cov3d, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_project_bwd: n < 0");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(means && scales && quats && viewmat && cov3d && radii && conics && compensation && v_xy &&
                  v_depth && v_conic && v_compensation && v_mean && v_scale && v_quat,
              "sfx_project_bwd: null buffer");
  project_bwd_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(
      n, means, scales, glob_scale, quats, viewmat, fx, fy, cov3d, radii, conics, compensation, v_xy, v_depth,
      v_conic, v_compensation, v_mean, v_scale, v_quat, v_cov2d, v_cov3d);
  return sfx::check_launch("sfx_project_bwd");
}

int sfx_isect_emit(int n, const float* xys, const float* depths, const int* radii, const int* cum_tiles_hit,
                   int tiles_x, int tiles_y, int block_width, int64_t* isect_ids, int32_t* gaussian_ids,
                   void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_isect_emit: n < 0");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_isect_emit: block_width must be in (1,16]");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(xys && depths && radii && cum_tiles_hit && isect_ids && gaussian_ids, "sfx_isect_emit: null buffer");
  isect_emit_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(
      n, xys, depths, radii, cum_tiles_hit, tiles_x, tiles_y, block_width, isect_ids, gaussian_ids, 0, INT_MAX);
  return sfx::check_launch("sfx_isect_emit");
}

int sfx_tile_bins(int num_isect, const int64_t* isect_ids_sorted, int num_tiles, int* tile_bins, void* stream) {
  SFX_REQUIRE(num_isect >= 0 && num_tiles > 0, "sfx_tile_bins: bad sizes");
  SFX_REQUIRE(tile_bins, "sfx_tile_bins: null tile_bins");
  hipStream_t st = sfx::as_stream(stream);
  hipMemsetAsync(tile_bins, 0, sizeof(int) * 2 * (size_t)num_tiles, st);
  if (num_isect > 0) {
    SFX_REQUIRE(isect_ids_sorted, "sfx_tile_bins: null isect ids");
    tile_bins_kernel<<<sfx::ceil_div(num_isect, 256), 256, 0, st>>>(num_isect, isect_ids_sorted, tile_bins);
  }
  return sfx::check_launch("sfx_tile_bins");
}

int sfx_rasterize_fwd(int tiles_x, int tiles_y, int block_width, int img_h, int img_w, const int32_t* gids_sorted,
                      const int* tile_bins, const float* xys, const float* conics, const float* colors,
                      const float* opacity, const float* background, float* final_Ts, int* final_idx,
                      float* out_img, float* out_alpha, void* stream) {
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_rasterize_fwd: block_width must be in (1,16]");
  SFX_REQUIRE(tiles_x == (img_w + block_width - 1) / block_width && tiles_y == (img_h + block_width - 1) / block_width,
              "sfx_rasterize_fwd: tile bounds do not match the image size");
  SFX_REQUIRE(tile_bins && xys && conics && colors && opacity && background && final_Ts && final_idx && out_img,
              "sfx_rasterize_fwd: null buffer");
  dim3 grid(tiles_x, tiles_y);
  rasterize_fwd_kernel<<<grid, block_width * block_width, 0, sfx::as_stream(stream)>>>(
      tiles_x, tiles_y, block_width, img_h, img_w, gids_sorted, tile_bins, xys, conics, colors, opacity, background,
      final_Ts, final_idx, out_img, out_alpha, 0);
  return sfx::check_launch("sfx_rasterize_fwd");
}

int sfx_rasterize_bwd(int tiles_x, int tiles_y, int block_width, int img_h, int img_w, const int32_t* gids_sorted,
                      const int* tile_bins, const float* xys, const float* conics, const float* colors,
                      const float* opacity, const float* background, const float* final_Ts, const int* final_idx,
                      const float* v_out, const float* v_out_alpha, float* v_xy, float* v_xy_abs, float* v_conic,
                      float* v_rgb, float* v_opacity, void* stream) {
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_rasterize_bwd: block_width must be in (1,16]");
  SFX_REQUIRE(tiles_x == (img_w + block_width - 1) / block_width && tiles_y == (img_h + block_width - 1) / block_width,
              "sfx_rasterize_bwd: tile bounds do not match the image size");
  SFX_REQUIRE(tile_bins && xys && conics && colors && opacity && background && final_Ts && final_idx && v_out &&
                  v_xy && v_conic && v_rgb && v_opacity,
              "sfx_rasterize_bwd: null buffer");
  dim3 grid(tiles_x, tiles_y);
  rasterize_bwd_kernel<<<grid, block_width * block_width, 0, sfx::as_stream(stream)>>>(
      tiles_x, tiles_y, block_width, img_h, img_w, gids_sorted, tile_bins, xys, conics, colors, opacity, background,
      final_Ts, final_idx, v_out, v_out_alpha, v_xy, v_xy_abs, v_conic, v_rgb, v_opacity);
  return sfx::check_launch("sfx_rasterize_bwd");
}

// ---- batched views (eval path of rasterize_gaussians_to_multiimgs) --------------------------------------
// All V cameras share the intrinsics / image size (the reference's cameras dict); per-view records are laid
// out view-major ([V, n, ...]); intersections of all views are sorted once (tile ids offset by view * T).
int sfx_render_prep_project_views(int n, int views, int num_bases, const float* means, long long ld_means,
                                  const float* log_scales, long long ld_scales, const float* quats_raw,
                                  long long ld_quats, const float* opac_logit, long long ld_opac,
                                  const float* features_dc, long long ld_dc, const float* features_rest,
                                  long long ld_rest, const float* camera_to_worlds, float fx, float fy, float cx,
                                  float cy, int img_h, int img_w, int block_width, float* rgbs, float* opacities,
                                  float* xys, float* depths, int* radii, float* conics, int* num_tiles_hit,
                                  float* records, void* stream) {
  SFX_REQUIRE(n >= 0 && views >= 1 && views <= 65535, "sfx_render_prep_project_views: bad sizes");
  SFX_REQUIRE((long long)n * views < (1ll << 31), "sfx_render_prep_project_views: views * n must fit int32");
  SFX_REQUIRE(num_bases == 1 || num_bases == 4 || num_bases == 9 || num_bases == 16 || num_bases == 25,
              "sfx_render_prep_project_views: num_bases must be a square in {1,4,9,16,25}");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_render_prep_project_views: block_width must be in (1,16]");
  SFX_REQUIRE(img_h > 0 && img_w > 0, "sfx_render_prep_project_views: empty image");
  SFX_REQUIRE(camera_to_worlds, "sfx_render_prep_project_views: null cameras");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(means && log_scales && quats_raw && opac_logit && features_dc && (num_bases == 1 || features_rest) &&
                  rgbs && opacities && xys && depths && radii && conics && num_tiles_hit,
              "sfx_render_prep_project_views: null buffer");
  launch_prep(n, views, num_bases, means, log_scales, quats_raw, opac_logit, features_dc, features_rest,
              PrepStrides{ld_means, ld_scales, ld_quats, ld_opac, ld_dc, ld_rest}, camera_to_worlds, fx, fy, cx, cy,
              img_h, img_w, block_width, nullptr, rgbs, opacities, xys, depths, radii, conics, num_tiles_hit,
              sfx::as_stream(stream), records);
  return sfx::check_launch("sfx_render_prep_project_views");
}

int sfx_isect_emit_views(int n_total, int n_per_view, const float* xys, const float* depths, const int* radii,
                         const int* cum_tiles_hit, int tiles_x, int tiles_y, int block_width, int64_t* isect_ids,
                         int32_t* gaussian_ids, long long capacity, void* stream) {
  SFX_REQUIRE(n_total >= 0 && n_per_view > 0 && n_total % n_per_view == 0, "sfx_isect_emit_views: bad sizes");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_isect_emit_views: block_width must be in (1,16]");
  if (n_total == 0) return SFX_OK;
  SFX_REQUIRE(xys && depths && radii && cum_tiles_hit && isect_ids && gaussian_ids,
              "sfx_isect_emit_views: null buffer");
  isect_emit_kernel<<<sfx::ceil_div(n_total, 256), 256, 0, sfx::as_stream(stream)>>>(
      n_total, xys, depths, radii, cum_tiles_hit, tiles_x, tiles_y, block_width, isect_ids, gaussian_ids, n_per_view,
      (int)(capacity < INT_MAX ? capacity : INT_MAX));
  return sfx::check_launch("sfx_isect_emit_views");
}

int sfx_rasterize_fwd_views(int views, int tiles_x, int tiles_y, int block_width, int img_h, int img_w,
                            const int32_t* gids_sorted, const int* tile_bins, const float* xys, const float* conics,
                            const float* colors, const float* opacity, const float* background, int clamp_max1,
                            float* final_Ts, int* final_idx, float* out_img, float* out_alpha, void* stream) {
  SFX_REQUIRE(views >= 1 && views <= 65535, "sfx_rasterize_fwd_views: bad view count");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_rasterize_fwd_views: block_width must be in (1,16]");
  SFX_REQUIRE(tiles_x == (img_w + block_width - 1) / block_width && tiles_y == (img_h + block_width - 1) / block_width,
              "sfx_rasterize_fwd_views: tile bounds do not match the image size");
  SFX_REQUIRE(tile_bins && xys && conics && colors && opacity && background && final_Ts && final_idx && out_img,
              "sfx_rasterize_fwd_views: null buffer");
  dim3 grid(tiles_x, tiles_y, views);
  rasterize_fwd_kernel<<<grid, block_width * block_width, 0, sfx::as_stream(stream)>>>(
      tiles_x, tiles_y, block_width, img_h, img_w, gids_sorted, tile_bins, xys, conics, colors, opacity, background,
      final_Ts, final_idx, out_img, out_alpha, clamp_max1);
  return sfx::check_launch("sfx_rasterize_fwd_views");
}

int sfx_pack_raster_records(int n, const float* xys, const float* conics, const float* colors, const float* opacity,
                            float* records, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_pack_raster_records: n < 0");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(xys && conics && colors && opacity && records, "sfx_pack_raster_records: null buffer");
  SFX_REQUIRE((reinterpret_cast<uintptr_t>(records) & 15) == 0, "sfx_pack_raster_records: records not 16-byte aligned");
  pack_raster_records_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(
      n, xys, conics, colors, opacity, reinterpret_cast<float4*>(records));
  return sfx::check_launch("sfx_pack_raster_records");
}

int sfx_rasterize_fwd_views_packed(int views, int tiles_x, int tiles_y, int block_width, int img_h, int img_w,
                                   const int32_t* gids_sorted, const int* tile_bins, const float* records,
                                   const float* background, int clamp_max1, float* final_Ts, int* final_idx,
                                   float* out_img, float* out_alpha, void* stream) {
  SFX_REQUIRE(views >= 1 && views <= 65535, "sfx_rasterize_fwd_views_packed: bad view count");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_rasterize_fwd_views_packed: block_width must be in (1,16]");
  SFX_REQUIRE(tiles_x == (img_w + block_width - 1) / block_width && tiles_y == (img_h + block_width - 1) / block_width,
              "sfx_rasterize_fwd_views_packed: tile bounds do not match the image size");
  SFX_REQUIRE(tile_bins && records && background && final_Ts && final_idx && out_img,
              "sfx_rasterize_fwd_views_packed: null buffer");
  SFX_REQUIRE((reinterpret_cast<uintptr_t>(records) & 15) == 0, "sfx_rasterize_fwd_views_packed: records alignment");
  dim3 grid(tiles_x, tiles_y, views);
  rasterize_fwd_packed_kernel<<<grid, block_width * block_width, 0, sfx::as_stream(stream)>>>(
      tiles_x, tiles_y, block_width, img_h, img_w, gids_sorted, tile_bins, reinterpret_cast<const float4*>(records),
      background, final_Ts, final_idx, out_img, out_alpha, clamp_max1);
  return sfx::check_launch("sfx_rasterize_fwd_views_packed");
}

int sfx_isect_count_cull_views(int n_total, int n_per_view, const float* xys, const float* conics,
                               const float* opacities, const int* radii, int tiles_x, int tiles_y, int block_width,
                               int img_h, int img_w, int* num_tiles_kept, void* stream) {
  SFX_REQUIRE(n_total >= 0 && n_per_view > 0 && n_total % n_per_view == 0, "sfx_isect_count_cull_views: bad sizes");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_isect_count_cull_views: block_width must be in (1,16]");
  SFX_REQUIRE(tiles_x == (img_w + block_width - 1) / block_width && tiles_y == (img_h + block_width - 1) / block_width,
              "sfx_isect_count_cull_views: tile bounds do not match the image size");
  if (n_total == 0) return SFX_OK;
  SFX_REQUIRE(xys && conics && opacities && radii && num_tiles_kept, "sfx_isect_count_cull_views: null buffer");
  isect_count_cull_kernel<<<sfx::ceil_div(n_total, 256), 256, 0, sfx::as_stream(stream)>>>(
      n_total, n_per_view, xys, conics, opacities, radii, tiles_x, tiles_y, block_width, img_h, img_w, num_tiles_kept);
  return sfx::check_launch("sfx_isect_count_cull_views");
}

int sfx_isect_emit_cull_views(int n_total, int n_per_view, const float* xys, const float* conics,
                              const float* opacities, const float* depths, const int* radii, const int* cum_tiles_hit,
                              int tiles_x, int tiles_y, int block_width, int img_h, int img_w, int64_t* isect_ids,
                              int32_t* gaussian_ids, const int* rank, long long capacity, void* stream) {
  SFX_REQUIRE(n_total >= 0 && n_per_view > 0 && n_total % n_per_view == 0, "sfx_isect_emit_cull_views: bad sizes");
  SFX_REQUIRE(block_width > 1 && block_width <= 16, "sfx_isect_emit_cull_views: block_width must be in (1,16]");
  SFX_REQUIRE(tiles_x == (img_w + block_width - 1) / block_width && tiles_y == (img_h + block_width - 1) / block_width,
              "sfx_isect_emit_cull_views: tile bounds do not match the image size");
  if (n_total == 0) return SFX_OK;
  SFX_REQUIRE(xys && conics && opacities && depths && radii && cum_tiles_hit && isect_ids && gaussian_ids,
              "sfx_isect_emit_cull_views: null buffer");
  isect_emit_cull_kernel<<<sfx::ceil_div(n_total, 256), 256, 0, sfx::as_stream(stream)>>>(
      n_total, n_per_view, xys, conics, opacities, depths, radii, cum_tiles_hit, tiles_x, tiles_y, block_width, img_h,
      img_w, isect_ids, gaussian_ids, rank, (int)(capacity < INT_MAX ? capacity : INT_MAX));
  return sfx::check_launch("sfx_isect_emit_cull_views");
}

int sfx_invert_permutation(long long n, const int* perm, int* inv, void* stream) {
  SFX_REQUIRE(n >= 0 && n < (1ll << 31), "sfx_invert_permutation: n out of range");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(perm && inv && perm != inv, "sfx_invert_permutation: null or aliased buffer");
  invert_perm_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, perm, inv);
  return sfx::check_launch("sfx_invert_permutation");
}

int sfx_depth_keys(long long n, const float* depths, uint64_t* keys, void* stream) {
  SFX_REQUIRE(n >= 0, "sfx_depth_keys: n < 0");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(depths && keys, "sfx_depth_keys: null buffer");
  depth_keys_kernel<<<sfx::ceil_div(n, 256), 256, 0, sfx::as_stream(stream)>>>(n, depths, keys);
  return sfx::check_launch("sfx_depth_keys");
}

int sfx_rasterize_fwd_views_quad(int views, int tiles_x, int tiles_y, int block_width, int img_h, int img_w,
                                 const int32_t* gids_sorted, const int* tile_bins, const float* records,
                                 const float* background, int clamp_max1, float* final_Ts, int* final_idx,
                                 float* out_img, float* out_alpha, void* stream) {
  SFX_REQUIRE(views >= 1 && views <= 65535, "sfx_rasterize_fwd_views_quad: bad view count");
  SFX_REQUIRE(block_width == 16, "sfx_rasterize_fwd_views_quad: block_width must be 16");
  SFX_REQUIRE(tiles_x == (img_w + 15) / 16 && tiles_y == (img_h + 15) / 16,
              "sfx_rasterize_fwd_views_quad: tile bounds do not match the image size");
  SFX_REQUIRE(tile_bins && records && background && final_Ts && final_idx && out_img,
              "sfx_rasterize_fwd_views_quad: null buffer");
  SFX_REQUIRE((reinterpret_cast<uintptr_t>(records) & 15) == 0, "sfx_rasterize_fwd_views_quad: records alignment");
  dim3 grid(tiles_x, tiles_y, views);
  rasterize_fwd_quad_kernel<<<grid, 256, 0, sfx::as_stream(stream)>>>(
      tiles_x, tiles_y, img_h, img_w, gids_sorted, tile_bins, reinterpret_cast<const float4*>(records), background,
      final_Ts, final_idx, out_img, out_alpha, clamp_max1);
  return sfx::check_launch("sfx_rasterize_fwd_views_quad");
}

int sfx_rasterize_bwd_quad(int tiles_x, int tiles_y, int block_width, int img_h, int img_w, const int32_t* gids_sorted,
                           const int* tile_bins, const float* xys, const float* conics, const float* colors,
                           const float* opacity, const float* background, const float* final_Ts, const int* final_idx,
                           const float* v_out, const float* v_out_alpha, float* v_xy, float* v_xy_abs, float* v_conic,
                           float* v_rgb, float* v_opacity, void* stream) {
  SFX_REQUIRE(block_width == 16, "sfx_rasterize_bwd_quad: block_width must be 16");
  SFX_REQUIRE(tiles_x == (img_w + 15) / 16 && tiles_y == (img_h + 15) / 16,
              "sfx_rasterize_bwd_quad: tile bounds do not match the image size");
  SFX_REQUIRE(tile_bins && xys && conics && colors && opacity && background && final_Ts && final_idx && v_out &&
                  v_xy && v_conic && v_rgb && v_opacity,
              "sfx_rasterize_bwd_quad: null buffer");
  dim3 grid(tiles_x, tiles_y);
  rasterize_bwd_quad_kernel<<<grid, 256, 0, sfx::as_stream(stream)>>>(
      tiles_x, tiles_y, img_h, img_w, gids_sorted, tile_bins, xys, conics, colors, opacity, background, final_Ts,
      final_idx, v_out, v_out_alpha, v_xy, v_xy_abs, v_conic, v_rgb, v_opacity);
  return sfx::check_launch("sfx_rasterize_bwd_quad");
}

}  // extern "C"
