/*
 * libsfx -- MI355X-native (gfx950) kernels for the SplatFormer refine+render
 * hot path.  Plain C ABI: caller-owned device buffers (any allocator; the
 * Python host side uses torch), an explicit hipStream_t passed as `void*`,
 * `int` status (0 = ok, <0 = error) and a thread-local message from
 * sfx_last_error().  Every entry point is stateless and reentrant; all
 * launches are asynchronous on `stream`.  No entry point syncs the host.
 *
 * Each function names the reference interface it replaces.  The gsplat and
 * Pointcept/spconv/torch_scatter call sites are the reference's, the
 * algorithms are the (un-vendored) dependencies' -- see DESIGN.md.
 */
#ifndef SFX_H_
#define SFX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFX_OK 0
#define SFX_ERR_INVALID -1
#define SFX_ERR_HIP -2
#define SFX_ERR_WORKSPACE -3

/* ---- library ------------------------------------------------------------ */
int sfx_abi_version(void);
const char* sfx_last_error(void);

/* ---- device primitives --------------------------------------------------- */
/* int32/int64 scan (inclusive != 0 -> inclusive).  `total` (optional, device)
 * receives the grand total.  Replaces torch.cumsum(num_tiles_hit, dtype=int32)
 * inside gsplat rasterize_gaussians (called at utils/gs_utils.py:96). */
size_t sfx_scan_workspace_bytes(long long n);
int sfx_scan_i32(long long n, const int32_t* in, int32_t* out, int inclusive, void* ws, size_t ws_bytes,
                 int32_t* total, void* stream);
int sfx_scan_i64(long long n, const int64_t* in, int64_t* out, int inclusive, void* ws, size_t ws_bytes,
                 int64_t* total, void* stream);

/* Stable LSD radix sort of (u64 key, i32 value) pairs on key bits
 * [begin_bit, end_bit).  vals_in == NULL sorts positions (argsort).
 * Replaces torch.sort(isect_ids) in gsplat bin_and_sort_gaussians
 * (utils/gs_utils.py:96) and torch.argsort(code) / torch.sort(cluster) in
 * Pointcept serialization/pooling (models/pointtransformer_v3.py:380, :290). */
size_t sfx_sort_workspace_bytes(long long n);
int sfx_sort_pairs_u64(long long n, const uint64_t* keys_in, const int32_t* vals_in, uint64_t* keys_out,
                       int32_t* vals_out, int begin_bit, int end_bit, void* ws, size_t ws_bytes, void* stream);

/* ---- render: gsplat v0.1.11 boundary (utils/gs_utils.py:78, :82-95, :96-109) */
/* gsplat.spherical_harmonics(degrees_to_use, viewdirs[N,3], coeffs[N,K,3]) -> colors[N,3]  (gs_utils.py:78) */
int sfx_sh_fwd(int n, int num_bases, int degrees_to_use, const float* viewdirs, const float* coeffs, float* colors,
               void* stream);
int sfx_sh_bwd(int n, int num_bases, int degrees_to_use, const float* viewdirs, const float* v_colors,
               float* v_coeffs, void* stream);

/* gsplat.project_gaussians(means3d, scales, glob_scale, quats(w,x,y,z), viewmat[3x4 row-major], fx, fy, cx, cy,
 *                          img_height, img_width, block_width, clip_thresh)  (gs_utils.py:82-95)
 * -> xys[N,2], depths[N], radii[N], conics[N,3], compensation[N], num_tiles_hit[N], cov3d[N,6] */
int sfx_project_fwd(int n, const float* means, const float* scales, float glob_scale, const float* quats,
                    const float* viewmat, float fx, float fy, float cx, float cy, int img_h, int img_w,
                    int block_width, float clip_thresh, float* xys, float* depths, int* radii, float* conics,
                    float* compensation, int* num_tiles_hit, float* cov3d, void* stream);
/* autograd backward of project_gaussians; v_cov2d / v_cov3d optional */
int sfx_project_bwd(int n, const float* means, const float* scales, float glob_scale, const float* quats,
                    const float* viewmat, float fx, float fy, const float* cov3d, const int* radii,
                    const float* conics, const float* compensation, const float* v_xy, const float* v_depth,
                    const float* v_conic, const float* v_compensation, float* v_mean, float* v_scale,
                    float* v_quat, float* v_cov2d, float* v_cov3d, void* stream);

/* Fused eval-path glue + SH + projection: utils/gs_utils.py:32-95 in one pass
 * (camera_to_world [3x4|4x4 row-major, OpenGL] -> viewmat_out[3x4]; exp(scales),
 * normalised quats, sigmoid(opacities), SH colours, project_gaussians). */
int sfx_render_prep_project(int n, int num_bases, const float* means, const float* log_scales,
                            const float* quats_raw, const float* opac_logit, const float* features_dc,
                            const float* features_rest, const float* camera_to_world, float fx, float fy, float cx,
                            float cy, int img_h, int img_w, int block_width, float* viewmat_out, float* rgbs,
                            float* opacities, float* xys, float* depths, int* radii, float* conics,
                            int* num_tiles_hit, void* stream);

/* gsplat map_gaussian_to_intersects: key = tile_id << 32 | bits(depth), val = gaussian id */
int sfx_isect_emit(int n, const float* xys, const float* depths, const int* radii, const int* cum_tiles_hit,
                   int tiles_x, int tiles_y, int block_width, int64_t* isect_ids, int32_t* gaussian_ids,
                   void* stream);
/* gsplat get_tile_bin_edges: tile_bins[num_tiles][2] = [start, end) */
int sfx_tile_bins(int num_isect, const int64_t* isect_ids_sorted, int num_tiles, int* tile_bins, void* stream);

/* gsplat rasterize_forward (3-channel): out_img[H,W,3], final_Ts[H,W], final_idx[H,W], out_alpha[H,W] (optional,
 * = 1 - final_Ts as returned by rasterize_gaussians(..., return_alpha=True)) */
int sfx_rasterize_fwd(int tiles_x, int tiles_y, int block_width, int img_h, int img_w, const int32_t* gids_sorted,
                      const int* tile_bins, const float* xys, const float* conics, const float* colors,
                      const float* opacity, const float* background, float* final_Ts, int* final_idx,
                      float* out_img, float* out_alpha, void* stream);
/* gsplat rasterize_backward_kernel; outputs are accumulated (+=) with float atomics: zero them first.
 * v_out_alpha and v_xy_abs may be NULL. */
int sfx_rasterize_bwd(int tiles_x, int tiles_y, int block_width, int img_h, int img_w, const int32_t* gids_sorted,
                      const int* tile_bins, const float* xys, const float* conics, const float* colors,
                      const float* opacity, const float* background, const float* final_Ts, const int* final_idx,
                      const float* v_out, const float* v_out_alpha, float* v_xy, float* v_xy_abs, float* v_conic,
                      float* v_rgb, float* v_opacity, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SFX_H_ */
