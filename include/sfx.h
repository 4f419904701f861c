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
 * inside gsplat rasterize_gaussians (called at utils/gs_utils.py:96).
 * (ABI v11) int32: one single-pass launch with decoupled look-back on a
 * library-owned ticket + tile-word area per (device, stream), epoch-tagged so
 * it needs no reset between scans (`ws` is unused by the int32 form and may be
 * NULL / 0); in place (in == out) allowed.  The first scan on a stream (or a
 * larger one) allocates the area (hipMalloc + stream-ordered zeroing; growing it
 * synchronises the stream): make one scan of the largest size before capturing
 * scans or sorts into a HIP graph. */
size_t sfx_scan_workspace_bytes(long long n);
/* (ABI v12) Look-back waits on this stream's area that hit the spin cap (each one a wrong scan / radix prefix,
 * never a hang) since the area was allocated; -1 when the stream has no area.  Synchronises the stream. */
long long sfx_lookback_timeouts(void* stream);
/* (ABI v12) Free this stream's look-back area after its pending work (call before destroying a stream that
 * scanned or sorted; a later scan on the stream allocates a new one). */
int sfx_lookback_release(void* stream);
int sfx_scan_i32(long long n, const int32_t* in, int32_t* out, int inclusive, void* ws, size_t ws_bytes,
                 int32_t* total, void* stream);
int sfx_scan_i64(long long n, const int64_t* in, int64_t* out, int inclusive, void* ws, size_t ws_bytes,
                 int64_t* total, void* stream);

/* Stable LSD radix sort of (u64 key, i32 value) pairs on key bits
 * [begin_bit, end_bit).  vals_in == NULL sorts positions (argsort).
 * Replaces torch.sort(isect_ids) in gsplat bin_and_sort_gaussians
 * (utils/gs_utils.py:96) and torch.argsort(code) / torch.sort(cluster) in
 * Pointcept serialization/pooling (models/pointtransformer_v3.py:380, :290).
 * (ABI v11) per 8-bit pass: tile histograms, one single-pass look-back scan
 * (on the stream's library-owned area, as sfx_scan_i32), stable scatter. */
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
 * normalised quats, sigmoid(opacities), SH colours, project_gaussians).  Each attribute is read with its
 * own row stride (elements), so the packed [N,23] refined-Gaussian record of the heads can be rendered
 * in place; features_rest rows hold (num_bases-1)*3 coefficients. */
int sfx_render_prep_project(int n, int num_bases, const float* means, long long ld_means, const float* log_scales,
                            long long ld_scales, const float* quats_raw, long long ld_quats, const float* opac_logit,
                            long long ld_opac, const float* features_dc, long long ld_dc, const float* features_rest,
                            long long ld_rest, const float* camera_to_world, float fx, float fy, float cx,
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

/* Eval-path rasterizer over packed records (round 2): sfx_pack_raster_records writes one record per projected
 * Gaussian, r0 = (x, y, opacity, conic.a), r1 = (conic.b, conic.c, r, g), r2 = (b, 0, 0, 0) -- (ABI v13) 16 floats
 * per record (64-byte stride; the fourth float4 is not written), records [n][16]; sfx_rasterize_fwd_views_packed is
 * sfx_rasterize_fwd_views over them (same outputs, bit for bit). */
int sfx_pack_raster_records(int n, const float* xys, const float* conics, const float* colors, const float* opacity,
                            float* records, void* stream);
int sfx_rasterize_fwd_views_packed(int views, int tiles_x, int tiles_y, int block_width, int img_h, int img_w,
                                   const int32_t* gids_sorted, const int* tile_bins, const float* records,
                                   const float* background, int clamp_max1, float* final_Ts, int* final_idx,
                                   float* out_img, float* out_alpha, void* stream);

/* ---- refiner: Pointcept PTv3 m1 + FeaturePredictor (models/pointtransformer_v3.py, feature_predictor.py) -- */
/* fp32 MFMA GEMM, Y = act((A' W^T + bias) * scale + shift) + R[ridx]; A' = A or, with gather_idx [M][S],
 * the concatenation of S gathered rows (SubMConv3d implicit GEMM).  act: 0 none, 1 GELU(erf), 2 ReLU,
 * 3 tanh, applied to columns < act_ncols (-1 = all).  Ypre (optional) receives the pre-residual value.
 * groups > 1 runs a grouped GEMM (block-diagonal heads) with the given per-group element strides.
 * out_row_idx[m] (optional) maps GEMM row m to its output row (residual_idx is indexed by output row).
 * Every operand must span < 2 GiB (raw buffer descriptors; out-of-range lanes read 0 / drop stores).
 * Replaces nn.Linear / BatchNorm1d(eval) / GELU / residual adds of Block, Embedding, SerializedPooling,
 * SerializedUnpooling and the FeaturePredictor heads (feature_predictor.py:74-94, :201-235), and
 * spconv.SubMConv3d (Block.cpe) through gather_idx. */
int sfx_linear(int M, int N, int K, const float* A, long long lda, const int* gather_idx, int num_segments,
               const float* W, long long ldw, const float* bias, const float* scale, const float* shift, int act,
               int act_ncols, const float* R, long long ldr, const int* residual_idx, float* Y, long long ldy,
               float* Ypre, long long ldypre, int groups, long long group_stride_A, long long group_stride_W,
               long long group_stride_bias, long long group_stride_Y, const int* out_row_idx, const float* rowscale,
               int pre_before_act, const unsigned long long* a_amax, unsigned a_tag,
               const unsigned long long* w_amax, unsigned w_tag, unsigned long long* y_amax, unsigned y_tag,
               const float* w_split, const float* w_inv, void* stream);

/* Pre-split weight for the fp16x2 GEMMs (ABI v5): dst has W's [rows x cols] shape in 4-byte units, contiguous;
 * every group of 4 consecutive elements of a row holds 4 fp16 h terms then 4 fp16 l terms of
 * W[n, k..k+3] * 2^e_n, where 2^e_n puts the row's largest magnitude in [2^14, 2^15); w_inv[n] = 2^-e_n.
 * cols and ld multiples of 4, buffers 16-byte aligned.  Passing (w_split, w_inv) of a weight to sfx_linear /
 * sfx_subm_conv / sfx_linear_bwd_data / sfx_subm_conv_bwd_data (split of the matrix passed as W / weight / Wt)
 * selects the fp16x2 kernel, which also scales every row of A' by its own power of two (chosen online from the
 * row's values), so no operand maxima are needed; NULL keeps the range-safe bf16x3 form. */
int sfx_weight_split(int rows, int cols, const float* w, long long ld, float* w_split, float* w_inv, void* stream);

/* fp16x2 operand maxima ("amax slots").  The GEMMs run K >= 64 products on split operands: fp16x2 by default
 * (a power-of-two scale per operand from an upper bound of its largest magnitude; SFX_GEMM_PREC=bf16x3 or fp32
 * select the other forms).  A slot is 64 unsigned long long sub-slots, zero-initialised by the caller once,
 * holding (tag << 32 | float bits) written with atomicMax; readers use the sub-slots carrying their tag.
 * a_amax / w_amax (may be NULL: the library then runs its own maxima pass) bound |A'| and |W| of a GEMM;
 * y_amax (may be NULL) receives max |Y| of a launch's outputs under y_tag (Stream-K is then not used).
 * sfx_amax_f32 writes max |X| of a [rows x cols] (row stride ld) matrix; sfx_ln_amax_bound writes the bound
 * sqrt(C-1) * max|gamma| + max|beta| of any LayerNorm output with those affine parameters. */
int sfx_amax_f32(int rows, int cols, const float* x, long long ld, unsigned long long* slot, unsigned tag,
                 void* stream);
int sfx_ln_amax_bound(int C, const float* gamma, const float* beta, unsigned long long* slot, unsigned tag,
                      void* stream);

/* Tuning / test hook: force the GEMM tile configuration (index into gemm.hip kCfgs, -1 = cost model) and
 * Stream-K (0 off, 1 on where legal, -1 = cost model) for every later sfx_linear / sfx_subm_conv call of the
 * process.  Eight-wave configurations apply only to split (K >= 64) launches. */
int sfx_gemm_force_config(int cfg, int stream_k);

/* Library operand-precision mode for every later GEMM launch issued by the calling host thread (ABI 14; per thread
 * since ABI 15 -- launches from other threads keep their own mode, default 0):
 *   0 (default) fp32-accurate: fp16x2 / bf16x3 split operands, three resp. six term products per block;
 *   1 reference precision, the class of the reference's fp16 autocast training (train.py:240,
 *     configs/train/default.gin:11): sfx_linear / sfx_subm_conv / sfx_linear_bwd_data and the SubM conv
 *     backward form only the leading fp16 product of each block (operands rounded to fp16 after the per-row
 *     power-of-two scaling, fp32 accumulation, fp32 outputs); so do the training MLP tail
 *     (sfx_block_mlp_train / sfx_block_mlp_bwd), sfx_window_attention_bwd and sfx_window_attention's fp16x2 form
 *     (its bf16x3 form, no qkv bound given: three bf16 products); sfx_linear_wgrad forms three bf16 products
 *     (16-bit significands).  The eval-only fused kernels (sfx_block_mlp, sfx_subm_cpe_ln, sfx_heads) ignore it.
 * Returns SFX_OK or an error for a mode other than 0 / 1; sfx_get_precision returns the current mode. */
int sfx_set_precision(int mode);
int sfx_get_precision(void);

/* ---- training (configs C/D): backward of the nn.Linear layers -------------------------------------
 * dX[M,K] (=|+=) rowscale[m] * (dY[M,N] W[N,K]) * act'(dact_pre[m,k]) for k < dact_ncols (-1 = all);
 * Wt = W^T stored [K, N] (ldwt); dact: 0 none, 1 GELU(erf) on the pre-activation, 2 ReLU, 3 tanh given
 * its output; rowscale = DropPath keep/(1-p) mask or NULL.  Autograd of F.linear + the activation that
 * feeds it (reference models run under train.py:240-289 `total_loss.backward()`). */
int sfx_linear_bwd_data(int M, int N, int K, const float* dY, long long ldy, const float* Wt, long long ldwt,
                        const float* rowscale, int dact, int dact_ncols, const float* dact_pre, long long ld_pre,
                        float* dX, long long lddx, int accumulate, const float* wt_split, const float* wt_inv,
                        void* stream);
/* dW[N,K] += dY[M,N]^T X[M,K]; db[N] += sum_m dY[m,:] (db may be NULL).  Accumulates (float atomics). */
int sfx_linear_wgrad(int M, int N, int K, const float* dY, long long ldy, const float* X, long long ldx, float* dW,
                     long long ldw, float* db, void* stream);
/* dst[c, r] = src[r, c] */
/* An empty kernel delimiting units of work in a rocprofv3 PMC / kernel trace (bench.py measure_traffic). */
int sfx_profile_marker(int tag, void* stream);

int sfx_transpose(int rows, int cols, const float* src, long long lds, float* dst, long long ldd, void* stream);
/* spconv SubMConv3d backward w.r.t. the input (the cpe.0 conv of every Block): dX[in] += dY[out] W_k over
 * the centre offset and every (in, out, k) pair of sfx_subm_pairs; weight_t = weight [Cout, 27*Cin]
 * transposed to [27*Cin, Cout]; centre_ws = 2n ints scratch; dX accumulates (float atomics). */
int sfx_subm_conv_bwd_data(int n, int cin, int cout, const float* dy, long long ldy, const int* nbr,
                           const float* weight_t, const int* pair_in, const int* pair_out, const int* pair_off_host,
                           int* centre_ws, float* dx, long long lddx, const float* wt_split, const float* wt_inv,
                           void* stream);
/* non-flash SerializedAttention backward (visualize.py:140-179 math): dout [N, C] = grad of the attention
 * output rows.  (ABI v13) attn_out [N, C] = the forward's output (Delta = dO . O), stats = workspace of
 * N * heads * 4 floats, 16-byte aligned (query pass -> key pass); every element of dqkv [N, 3C] is written.
 * Under SFX_ATTN_PREC=fp32 (the exact single-kernel backward) attn_out and stats are unused and dqkv must be
 * zero-filled (dK/dV accumulate across overlapping windows). */
int sfx_window_attention_bwd(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                             const int* order, const int* win, float scale, const float* attn_out, const float* dout,
                             float* dqkv, float* stats, void* stream);
/* (ABI v7) enable_flash=True backward (windows as sfx_window_attention_varlen): dqkv [N, 3C] zero-filled,
 * stats = workspace of N * heads * 2 floats (per-query log-sum-exp and dO.O). */
int sfx_window_attention_varlen_bwd(int num_windows, int max_window, int heads, int head_dim, int channels,
                                    const float* qkv, const int* order, const int* win3, float scale,
                                    const float* dout, float* dqkv, float* stats, void* stream);
/* nn.LayerNorm backward w.r.t. the input: dX = LN'(X) dY (+ dR) */
int sfx_layernorm_bwd(int M, int C, const float* X, long long ldx, const float* gamma, const float* dY,
                      long long ldgy, const float* dR, long long ldr, float eps, float* dX, long long lddx,
                      void* stream);
/* Block tail backward: dX1 = dX2 + LN1'(X1) dH ; dU = LN_cpe'(U) dX1   (rows of C contiguous floats) */
int sfx_cpe_ln_bwd(int M, int C, const float* U, const float* X1, const float* gamma_cpe, const float* gamma1,
                   const float* dX2, const float* dH, float eps, float* dX1, float* dU, void* stream);
/* train-mode nn.BatchNorm1d(eps 1e-3, momentum 0.01) [+ GELU]; SyncBatchNorm: all-reduce `sums` between the
 * reduce and the finalize/apply calls.  sums = double[2C]. */
size_t sfx_colsum2_workspace_bytes(int M, int C);
int sfx_bn_stats(int M, int C, const float* X, long long ldx, void* ws, size_t ws_bytes, double* sums, void* stream);
int sfx_bn_finalize(int C, double count, const double* sums, const float* gamma, const float* beta, float eps,
                    float momentum, float* running_mean, float* running_var, float* mean_out, float* rstd_out,
                    float* scale_out, float* shift_out, void* stream);
int sfx_affine_act(int M, int C, const float* X, long long ldx, const float* scale, const float* shift, int act,
                   const float* R, long long ldr, const int* ridx, float* Y, long long ldy, void* stream);
int sfx_bn_act_bwd_reduce(int M, int C, const float* X, long long ldx, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, int act, const float* dY, long long ldgy, void* ws,
                          size_t ws_bytes, double* sums, void* stream);
int sfx_bn_act_bwd_apply(int M, int C, const float* X, long long ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* beta, int act, const float* dY, long long ldgy,
                         const double* sums, double count, float* dX, long long lddx, int accumulate, void* stream);
/* SerializedPooling segment_csr(max) with arg-max (train) and its backward (dX rows pre-zeroed) */
int sfx_segment_max_arg(int m, int C, const int* idx_ptr, const int* sorted_idx, const float* X, float* Y, int* arg,
                        void* stream);
int sfx_segment_max_bwd(int m, int C, const float* dY, const int* arg, float* dX, void* stream);
/* SerializedUnpooling backward of feat[inverse]: Y[s] = sum of the rows of cluster s */
int sfx_segment_sum(int m, int C, const int* idx_ptr, const int* sorted_idx, const float* X, long long ldx, float* Y,
                    void* stream);
/* dX = dY * act'(pre) on cols < ncols (1 GELU pre-act, 2 ReLU, 3 tanh given its output) */
int sfx_act_bwd(int M, int N, const float* dY, long long ldgy, const float* pre, long long ldp, int act, int ncols,
                float* dX, long long lddx, void* stream);
/* (ABI v13) DropPath keep mask of n points (timm DropPath, pointtransformer_v3.py:145): out[i] = 1/keep or 0,
 * Bernoulli(keep) from a counter-based hash of (seed, i) -- deterministic for a given seed */
int sfx_drop_mask(long long n, float keep, unsigned long long seed, float* out, void* stream);
/* clip_grad_norm_(max_norm) + torch.optim.Adam (train.py:292-302, utils/optimizers.py) */
int sfx_sumsq(long long n, const float* x, double* out, void* stream);
int sfx_clip_coef(const double* sumsq, float max_norm, float* coef, float* norm_out, void* stream);
int sfx_adam_step(long long n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  const float* grad_scale, float lr, float beta1, float beta2, float eps, float weight_decay,
                  int step, void* stream);

/* nn.LayerNorm rows (C <= 512): Block.norm1 / norm2 */
int sfx_layernorm(int M, int C, const float* X, long long ldx, const float* gamma, const float* beta, float eps,
                  float* Y, long long ldy, void* stream);
/* Block tail of cpe + shortcut + norm1: X_out = X + LN_cpe(T); H = LN1(X_out)  (X_out may alias X) */
int sfx_cpe_residual_ln(int M, int C, const float* T, const float* X, const float* gamma_cpe, const float* beta_cpe,
                        const float* gamma1, const float* beta1, float eps, float* X_out, float* H, void* stream);
/* (ABI v6) the same with T = the centre output of sfx_subm_conv_partials plus, per row, the SubM pair partials
 * partials[pair_pos[row][k]] summed in ascending offset order k (pair_pos: sfx_subm_pair_pos; -1 entries skipped):
 * the conv without float atomics, bitwise reproducible.  C in {64, 96, 128, 256, 512}, 16-byte aligned rows.
 * (ABI v15) ldt = T's row stride: C, or 0 when T is the conv bias [C] alone and the pair lists carry the centre
 * offset (sfx_subm_pairs with_centre = 1: the centre's products are partial rows too, added at k = 13). */
int sfx_cpe_residual_ln_pairs(int M, int C, const float* T, long long ldt, const float* partials, const int* pair_pos,
                              long long num_pairs, const float* X, const float* gamma_cpe, const float* beta_cpe,
                              const float* gamma1, const float* beta1, float eps, float* X_out, float* H,
                              void* stream);
/* (ABI v16) sfx_cpe_residual_ln_pairs reading the compacted positions pair_cpos [M][32] of sfx_subm_pair_lists:
 * the same sums in the same order (absent offsets add +0 in both), ceil(max count / 8) groups of 8 row loads per wave
 * instead of 27 position and 27 row loads per row. */
int sfx_cpe_residual_ln_cpairs(int M, int C, const float* T, long long ldt, const float* partials,
                               const int* pair_cpos, long long num_pairs, const float* X, const float* gamma_cpe,
                               const float* beta_cpe, const float* gamma1, const float* beta1, float eps, float* X_out,
                               float* H, void* stream);
/* (ABI v15) sfx_cpe_residual_ln_pairs followed by the Block's qkv projection in one launch (eval, C in {64, 96, 128};
 * calflops.py:45-55): X_out = X + LN_cpe(T + pair partials); qkv [M][3C] = LN1(X_out) W^T + bias with
 * W = sfx_weight_split of the qkv weight [3C][C] (w_split, w_inv) -- the norm1 output never leaves the chip.
 * max |qkv| is published into amax_slot (tag; may be NULL) for sfx_window_attention's fp16x2 scale.  X_out != X. */
int sfx_cpe_ln_qkv_pairs(int M, int C, const float* T, long long ldt, const float* partials, const int* pair_pos,
                         long long num_pairs, const float* X, const float* gamma_cpe, const float* beta_cpe,
                         const float* gamma1, const float* beta1, float eps, float* X_out, const float* w_split,
                         const float* w_inv, const float* bias, float* qkv, unsigned long long* amax_slot,
                         unsigned tag, void* stream);

/* SerializedAttention (non-flash): windows win[w] = (key_start, query_start) over serialized positions,
 * qkv [N,3C] in point order, order [N] serialized->point; out[order[p]] for every query position p. */
int sfx_window_attention(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                         const int* order, const int* win, float scale, float* out,
                         const unsigned long long* qkv_amax, unsigned qkv_tag, void* stream);
/* (ABI v7) SerializedAttention with enable_flash=True (reference models/pointtransformer_v3.py:121-123: patch
 * 1024; Pointcept's flash branch cuts the padded sequence at cu_seqlens): win3[w] = (key_start, query_start,
 * key_count), key_count <= max_window <= 2^20 (a batch of n <= K points is one n-key window); online softmax over
 * 128-key blocks.  Same qkv / order / out layout and the same term forms as sfx_window_attention (fp16x2 when
 * qkv_amax bounds |qkv|, bf16x3 without, exact fp32 MFMA under SFX_ATTN_PREC=fp32). */
int sfx_window_attention_varlen(int num_windows, int max_window, int heads, int head_dim, int channels,
                                const float* qkv, const int* order, const int* win3, float scale, float* out,
                                const unsigned long long* qkv_amax, unsigned qkv_tag, void* stream);
/* (ABI v15) Fused attention + output projection + residual for the eval Block (calflops.py:51-69:
 * x = shortcut + proj(attn(norm1 x))): x2[r] = x1[r] + bias + W . concat_h(softmax(q_h k_h^T scale) v_h)[r] over the
 * non-flash windows of sfx_window_attention (same `win` table, order, scale), all heads of a window in one
 * workgroup, the per-head outputs never leaving the chip.  fp16x2 terms only: qkv_amax (required) bounds |qkv|;
 * w_split / w_inv = sfx_weight_split of the projection weight [C][C]; bias [C]; x1 [n][ldx1] and x2 [n][ldx2]
 * distinct, 16-byte aligned rows.  (channels, head_dim) in {(64, 32), (96, 24), (128, 16), (256, 16)}. */
int sfx_window_attention_proj(int num_windows, int window, int heads, int head_dim, int channels, const float* qkv,
                              const int* order, const int* win, float scale, const unsigned long long* qkv_amax,
                              unsigned qkv_tag, const float* w_split, const float* w_inv, const float* bias,
                              const float* x1, long long ldx1, float* x2, long long ldx2, void* stream);

/* Point.serialization: codes[R][n] = batch << 3*depth | enc_t(grid) for order types t0..t3 (0 z, 1 z-trans,
 * 2 hilbert, 3 hilbert-trans) and combined sort keys r << code_bits | code; finalize turns the argsort of
 * the keys into order[R][n] / inverse[R][n]. */
int sfx_serialize_keys(int n, const int* grid_coord, const int* batch, int depth, int num_orders, int t0, int t1,
                       int t2, int t3, int code_bits, int64_t* codes, uint64_t* keys, void* stream);
/* (ABI v12) Renumber a serialized point set by its first order (new point i = old point order[0][i]): codes,
 * orders and inverses [R][n] re-expressed in the new numbering, grid [n][3] int32 and coord [n][3] float gathered --
 * the refiner's stage-0 locality permutation (sfx_move_rows). */
int sfx_serialize_permute(int n, int num_orders, const int* order, const int* inverse, const int64_t* codes,
                          const int* grid, const float* coord, int64_t* codes_p, int* order_p, int* inverse_p,
                          int* grid_p, float* coord_p, void* stream);
int sfx_serialize_finalize(int n, int num_orders, const int* sorted_pos, int* order, int* inverse, void* stream);

/* SerializedPooling (reference models/pointtransformer_v3.py:290-299 -> upstream Pointcept), sort-free: the parent's serialized
 * orders already list every coarse cell's points contiguously (codes are hierarchical, code >> 3pd is the
 * pooled code), so run starts replace torch.unique(code[0] >> 3pd), torch.sort(cluster) and the pooled argsort.
 *   run_flags:   flags[r*n + j] = 1 where order row r's j-th point starts a run of equal code >> shift;
 *                inclusive-scan the R*n flags (sfx_scan_i32) into `pos`; every row must count the same m runs.
 *   assign_runs: row0 (the first order type): cluster id per point (pooling_inverse), CSR members
 *                (sorted_idx, idx_ptr[m+1]; members in row0 order), one head point per cluster.
 *   reorder:     order / inverse [R][m] of the pooled points for every row.
 *   gather:      pooled codes [R][m], grid >> pd, batch from the heads (keys may be NULL).
 * Then segment max (+BN affine +GELU) of the projected features and the mean of the coords. */
int sfx_pool_run_flags(int n, int num_orders, const int* order, const int64_t* codes, int shift, int* flags,
                       void* stream);
/* (ABI v15) counts[k] (k < nshift <= 8; host array `shifts`) = the number of runs of codes[order[j]] >> shifts[k]
 * along ONE serialized row (order, codes: row 0's [n]) = the sum of sfx_pool_run_flags' flags for that shift: every
 * pooling's cluster count from the stage-0 codes in one launch (plus a 4-byte memset) */
int sfx_pool_run_counts(int n, const int* order, const int64_t* codes, const int* shifts, int nshift, int* counts,
                        void* stream);
int sfx_pool_assign_runs(int n, int m, int row0, const int* order, const int* pos, const int* flags, int* cluster,
                         int* idx_ptr, int* head, int* sorted_idx, void* stream);
int sfx_pool_reorder(int n, int m, int num_orders, const int* order, const int* pos, const int* flags,
                     const int* cluster, int* new_order, int* new_inverse, void* stream);
int sfx_pool_gather(int m, int n, int num_orders, const int* head, const int64_t* codes, int pooling_depth,
                    const int* grid_coord, const int* batch, int code_bits, int64_t* new_codes, uint64_t* keys,
                    int* new_grid, int* new_batch, void* stream);
int sfx_segment_max_affine_act(int m, int C, const int* idx_ptr, const int* sorted_idx, const float* X,
                               const float* scale, const float* shift, int act, float* Y, void* stream);
int sfx_segment_mean(int m, int D, const int* idx_ptr, const int* sorted_idx, const float* X, float* Y,
                     void* stream);

/* spconv SubMConv3d indice pairs (indice_key=stage{s}): nbr[n][27], k = (dx+1)*9+(dy+1)*3+(dz+1), -1 absent,
 * duplicate voxels resolve to the lowest point index; mask[n] (optional) = bit k set iff nbr[.][k] >= 0,
 * mask_keys[n] (optional) the same mask widened to the u64 sort-key layout.
 * table_*: 2^log2cap scratch slots.  sfx_subm_permute reorders nbr/mask rows by a permutation (the
 * mask-sorted row order that keeps each GEMM tile's segment union small). */
int sfx_subm_table_log2(int n);
int sfx_subm_neighbors(int n, const int* grid_coord, const int* batch, int log2cap, unsigned long long* table_keys,
                       int* table_vals, int* nbr, unsigned* mask, unsigned long long* mask_keys, void* stream);
int sfx_subm_permute(int n, const int* perm, const int* nbr, const unsigned* mask, int* nbr_sorted,
                     unsigned* mask_sorted, void* stream);
/* Offset-major indice pairs (centre offset excluded, output rows ascending within an offset):
 * pair_in/pair_out [<= 26 n], pair_off[28] (device) = per-offset prefix of the pair counts.
 * (ABI v15) with_centre = 1: the centre offset k = 13 is listed too ([<= 27 n] entries) -- the eval conv then runs
 * as ONE pair launch (sfx_subm_conv_partials_pairs) whose centre products are partial rows like the others
 * (summed by sfx_cpe_residual_ln_pairs with ldt = 0); sfx_subm_conv / sfx_subm_conv_bwd_data take lists without it. */
size_t sfx_subm_pairs_workspace_bytes(int n);
int sfx_subm_pairs(int n, const int* nbr, void* ws, size_t ws_bytes, int* pair_in, int* pair_out, int* pair_off,
                   int with_centre, void* stream);
/* (ABI v6) inverted pair index: pair_pos[i][k] = index of pair (k, out = i) in pair_in/pair_out, -1 if none
 * (always -1 for the centre k = 13 unless the lists carry it); pair_off = the device pair_off of sfx_subm_pairs,
 * num_pairs = pair_off[27]. */
int sfx_subm_pair_pos(int n, long long num_pairs, const int* pair_out, const int* pair_off, int* pair_pos,
                      void* stream);
/* (ABI v16) sfx_subm_pairs' lists -- the same pair_in / pair_out / pair_off, bit for bit -- and, when pair_pos is not
 * null, sfx_subm_pair_pos's inverted index, in two passes over nbr: per-workgroup (256 points) pair counts of every
 * offset, one scan of those 27 * ceil(n / 256) counts, then each workgroup writes its pairs (wave ballots keep the
 * output rows ascending within an offset) and its rows of pair_pos.  No host value is needed (sfx_subm_pair_pos needs
 * num_pairs). */
size_t sfx_subm_pair_lists_workspace_bytes(int n);
int sfx_subm_pair_lists(int n, const int* nbr, void* ws, size_t ws_bytes, int* pair_in, int* pair_out, int* pair_off,
                        int* pair_pos, int* pair_cpos, int with_centre, void* stream);
/* pair_cpos (nullable, [n][32], 16-byte aligned): row i's present pair indices in ascending offset order, -1 after
 * them, their count in element 31 -- the compacted form sfx_cpe_residual_ln_cpairs reads. */
/* spconv SubMConv3d(Cin, Cout, 3, bias) forward on the pair lists: out = bias + x[nbr[:,13]] W_13^T (dense centre
 * GEMM, plain stores), then one fp32 MFMA launch over the 26 other offsets' gathered rows whose partial products
 * are atomically added into out (float atomics: summation order across offsets is not fixed).
 * weight [Cout,3,3,3,Cin]; pair_off_host = the 28 pair_off values copied to the host. */
int sfx_subm_conv(int n, int cin, int cout, const float* x, long long ldx, const int* nbr, const float* weight,
                  const float* bias, const int* pair_in, const int* pair_out, const int* pair_off_host, float* out,
                  long long ldo, const unsigned long long* x_amax, unsigned x_tag,
                  const unsigned long long* w_amax, unsigned w_tag, const float* w_split, const float* w_inv,
                  void* stream);
/* (ABI v6) atomic-free form: out = bias + the centre offset's product; the 26 other offsets' products are stored
 * as rows of partials [pair_off[27]][ldp] (row = pair index) for sfx_cpe_residual_ln_pairs to sum per output row
 * in a fixed offset order. */
int sfx_subm_conv_partials(int n, int cin, int cout, const float* x, long long ldx, const int* nbr,
                           const float* weight, const float* bias, const int* pair_in, const int* pair_out,
                           const int* pair_off_host, float* out, long long ldo, float* partials, long long ldp,
                           const float* w_split, const float* w_inv, void* stream);
/* (ABI v10) the pair launch of sfx_subm_conv_partials alone, for a caller that made the centre launch first (an
 * sfx_subm_conv_partials call with pair_in = NULL and 28 zero offsets) and only then waits for pair_off_host. */
int sfx_subm_conv_partials_pairs(int n, int cin, int cout, const float* x, long long ldx, const int* nbr,
                                 const float* weight, const float* bias, const int* pair_in, const int* pair_out,
                                 const int* pair_off_host, float* out, long long ldo, float* partials, long long ldp,
                                 const float* w_split, const float* w_inv, void* stream);

/* FeaturePredictor batchify (feature_predictor.py:134-156): strided attribute rows -> feat rows
 * [means,scales,opacities,quats,dc,rest], grid_coord = floor(means*res), optional atomic grid max. */
int sfx_gs_pack(int n, const float* means, long long ld_means, const float* scales, long long ld_scales,
                const float* opacities, long long ld_opacities, const float* quats, long long ld_quats,
                const float* features_dc, long long ld_dc, const float* features_rest, long long ld_rest,
                int rest_dim, float grid_resolution, float* feat, long long ld_feat, int* grid_coord, int* grid_max,
                void* stream);
/* Pointcept offset2batch */
int sfx_offsets_to_batch(int n, int B, const long long* offsets, int* batch, void* stream);
/* (ABI v12) Row moves by index, rows of `words` 32-bit words (leading dimensions in words): scatter = 0 gathers
 * dst[i] = src[idx[i]], scatter = 1 scatters dst[idx[i]] = src[i].  The refiner's stage-0 z-order row permutation
 * (PointTransformerV3Model reorder: the input Gaussians enter in file order; the backbone runs them in serialized
 * order so every stage-0 gather is local, and the features go back to file order before the heads). */
int sfx_move_rows(long long n, int words, const void* src, long long src_ld, const int* idx, void* dst,
                  long long dst_ld, int scatter, void* stream);

/* ---- batched views: the eval path of gs_utils.rasterize_gaussians_to_multiimgs (gs_utils.py:20-27) ------
 * V cameras with shared intrinsics: records laid out [V, n, ...]; intersections of all views sorted once
 * with tile ids offset by view * tiles; rasterizer grid (tiles_x, tiles_y, V); clamp_max1 = gs_utils.py:111. */
int sfx_render_prep_project_views(int n, int views, int num_bases, const float* means, long long ld_means,
                                  const float* log_scales, long long ld_scales, const float* quats_raw,
                                  long long ld_quats, const float* opac_logit, long long ld_opac,
                                  const float* features_dc, long long ld_dc, const float* features_rest,
                                  long long ld_rest, const float* camera_to_worlds, float fx, float fy, float cx,
                                  float cy, int img_h, int img_w, int block_width, float* rgbs, float* opacities,
                                  float* xys, float* depths, int* radii, float* conics, int* num_tiles_hit,
                                  float* records, void* stream);
/* (ABI v13) records (optional, [views * n][16]): also writes sfx_pack_raster_records' record of every
 * Gaussian-view (no separate packing pass) */
/* (ABI v15) capacity: the length of isect_ids / gaussian_ids; pairs whose prefix offset falls outside [0, capacity)
 * are dropped, so a wrong prefix (a look-back scan that reached its spin cap, sfx_lookback_timeouts) can give a
 * wrong list but never an out-of-bounds write (also sfx_isect_emit_cull_views) */
int sfx_isect_emit_views(int n_total, int n_per_view, const float* xys, const float* depths, const int* radii,
                         const int* cum_tiles_hit, int tiles_x, int tiles_y, int block_width, int64_t* isect_ids,
                         int32_t* gaussian_ids, long long capacity, void* stream);
int sfx_rasterize_fwd_views(int views, int tiles_x, int tiles_y, int block_width, int img_h, int img_w,
                            const int32_t* gids_sorted, const int* tile_bins, const float* xys, const float* conics,
                            const float* colors, const float* opacity, const float* background, int clamp_max1,
                            float* final_Ts, int* final_idx, float* out_img, float* out_alpha, void* stream);
/* (ABI v9) exact contribution culling for the eval path (replaces sfx_isect_emit_views + the tile counts of
 * sfx_render_prep_project_views; same reference call site gs_utils.py:96-109 -> gsplat bin_and_sort_gaussians):
 * a (Gaussian, tile) pair of gsplat's 3-sigma square is kept unless alpha < 1/255 at every pixel centre of the
 * tile (minimum of the conic over the tile, double precision, with a margin for the fp32 per-pixel rounding).
 * sfx_isect_count_cull_views writes the surviving tile count of every projected Gaussian into num_tiles_kept
 * (gsplat's own counts stay in sfx_render_prep_project_views' num_tiles_hit: its per-view emptiness decides the
 * empty-image branch); sfx_isect_emit_cull_views, over the inclusive scan of num_tiles_kept, writes the
 * survivors (a subsequence of gsplat's list).  sfx_rasterize_fwd_views_quad = sfx_rasterize_fwd_views_packed with one
 * 8x8 quadrant per wave and per-wave record lists (block_width 16); images / alphas / final T bit-identical to
 * the unculled path, final_idx indexes the culled list. */
int sfx_isect_count_cull_views(int n_total, int n_per_view, const float* xys, const float* conics,
                               const float* opacities, const int* radii, int tiles_x, int tiles_y, int block_width,
                               int img_h, int img_w, int* num_tiles_kept, void* stream);
int sfx_isect_emit_cull_views(int n_total, int n_per_view, const float* xys, const float* conics,
                              const float* opacities, const float* depths, const int* radii, const int* cum_tiles_hit,
                              int tiles_x, int tiles_y, int block_width, int img_h, int img_w, int64_t* isect_ids,
                              int32_t* gaussian_ids, const int* rank, long long capacity, void* stream);
/* (ABI v13) two-level intersection sort: keys[i] = the depth bits of depths[i] (u64).  Argsorting them (stable,
 * sfx_sort_pairs_u64 bits [0, 32)) gives `order`, sfx_invert_permutation its inverse `rank`;
 * sfx_isect_emit_cull_views with that rank (cum_tiles_hit = the inclusive scan of num_tiles_kept[order]) emits the
 * pairs depth-sorted, and a stable sort of bits [32, 32 + tile bits) alone then yields gsplat's (tile, depth) order
 * with its emission-order ties: the same list as a full 64-bit sort, with the depth passes run over Gaussian-views
 * instead of pairs.  rank = NULL: emission in index order. */
int sfx_depth_keys(long long n, const float* depths, uint64_t* keys, void* stream);
int sfx_invert_permutation(long long n, const int* perm, int* inv, void* stream);
int sfx_rasterize_fwd_views_quad(int views, int tiles_x, int tiles_y, int block_width, int img_h, int img_w,
                                 const int32_t* gids_sorted, const int* tile_bins, const float* records,
                                 const float* background, int clamp_max1, float* final_Ts, int* final_idx,
                                 float* out_img, float* out_alpha, void* stream);
/* (ABI v9) sfx_rasterize_bwd over a culled list (sfx_isect_emit_cull_views, single view) and the final_idx of
 * sfx_rasterize_fwd_views_quad: one 8x8 quadrant per wave with per-wave record lists; block_width 16.  Same
 * contract as sfx_rasterize_bwd (outputs accumulated with float atomics: zero them first). */
int sfx_rasterize_bwd_quad(int tiles_x, int tiles_y, int block_width, int img_h, int img_w, const int32_t* gids_sorted,
                           const int* tile_bins, const float* xys, const float* conics, const float* colors,
                           const float* opacity, const float* background, const float* final_Ts, const int* final_idx,
                           const float* v_out, const float* v_out_alpha, float* v_xy, float* v_xy_abs, float* v_conic,
                           float* v_rgb, float* v_opacity, void* stream);

/* ---- evaluation post-processing ------------------------------------------------------------------
 * Replaces train.py:104-113 `(x*255).to(torch.uint8)` of prediction (after the gs_utils.py:111
 * clamp(max=1), applied when clamp_pred != 0) and ground truth, feeding utils/metrics.py:89-91 psnr.
 * sums[img*3 + {0,1,2}] = exact sum(p^2), sum(g^2), sum(p*g) of the quantised values;
 * maxes[img*2 + {0,1}] = max(p), max(g) (the metrics.py:26-29 "divide by 255 if max > 1" rule).
 * Images are [num_images, elems_per_image] contiguous f32. */
int sfx_image_stats_u8(int num_images, long long elems_per_image, const float* pred, const float* gt,
                       int clamp_pred, unsigned long long* sums, int* maxes, void* stream);
/* SSIM per image (utils/metrics.py:93-135: 11x11 Gaussian window sigma 1.5, zero padding, C1 = 0.01^2,
 * C2 = 0.03^2, mean of the SSIM map over channels and pixels).  img1/img2: [num_images][height][width][channels]
 * fp32 (HWC, as rendered); window: the 121 fp32 taps of the reference's 2-D window (row-major); out: [num_images].
 * quantize_u8 = 1 evaluates the uint8 images the evaluation loop scores ((x*255) truncated, img1 clamped to <= 1,
 * then /255: train.py:104-113, metrics.py:26-29); 0 uses the values as given. */
size_t sfx_ssim_workspace_bytes(int num_images, int height, int width, int channels);
int sfx_ssim(int num_images, int height, int width, int channels, const float* img1, const float* img2,
             const float* window, int quantize_u8, float* out, void* ws, size_t ws_bytes, void* stream);

/* Point-cloud downsampling experiments (reference models/pcd_downsampling_methods.py; FeaturePredictor
 * additional_info["downsample"], models/feature_predictor.py:159-196).
 * sfx_voxel_keys: voxel_downsample's ids (:96-100) as sort keys: floor(p / voxel_size) in fp32, the int32 hash
 *   x*1000000 + y*1000 + z, biased (id ^ 0x80000000) so unsigned order = signed order.  points: [n][ld] f32.
 * sfx_nn1: out[i] = index of the nearest of the m reference points to query i (float64 squared distance of the
 *   f32 coordinates, lowest index on ties) -- the sklearn NearestNeighbors(n_neighbors=1) queries of
 *   fps_knn_downsample (:45-48) and knn_map_back (:192-195).  queries [n][3], refs [m][3] f32 contiguous.
 * sfx_fps: furthest_point_sampling (:8-26) from `start` (the caller's torch.randint draw): out[m] indices;
 *   dist_ws: n floats. */
int sfx_voxel_keys(int n, const float* points, long long ld, float voxel_size, unsigned long long* keys,
                   void* stream);
int sfx_nn1(int n, int m, const float* queries, const float* refs, int* out, void* stream);
int sfx_fps(int n, int m, const float* xyz, int start, int* out, float* dist_ws, void* stream);

/* (ABI v8) Fused Block MLP tail, eval (reference Block.forward restated in calflops.py:72-82: norm2 -> mlp ->
 * + shortcut; MLP = Linear(C, 4C) -> GELU(erf) -> Linear(4C, C)):  Y = X + fc2(GELU(fc1(LN(X)))), one launch, the
 * LayerNorm output and the [M, 4C] hidden activation stay on chip.  fp32-accurate (fp16x2 MFMA terms with
 * power-of-two row scales, fp32 accumulation).  C in {64, 96, 128, 256}.
 * sfx_mlp_pack (once per weight version): w1 [4C][C], b1 [4C], w2 [C][4C], b2 [C], gamma / beta [C] (torch
 *   Linear / LayerNorm layouts, contiguous) -> `stream` (sfx_mlp_stream_floats(C) floats: the pre-split weights
 *   in the kernel's LDS-DMA slab order) and `params` (sfx_mlp_params_floats(C) floats); workspace: 9C ints.
 * sfx_block_mlp: X [M][ldx], Y [M][ldy] (distinct buffers), 16-byte aligned rows; eps = the LayerNorm eps.
 * At C >= 128 (and in the training entries below) a launch whose last round of workgroups is at most half full
 * runs that round as hidden-chunk partials + a fixed-order combine (bitwise reproducible) in a library-owned
 * scratch buffer per (device, stream), reused in stream order (SFX_MLP_SPLIT=0: one launch).  The buffer grows
 * on the first call that needs more (synchronising that stream once): under HIP graph capture, run the entry
 * once at the captured sizes before capturing. */
size_t sfx_mlp_stream_floats(int C);
size_t sfx_mlp_params_floats(int C);
int sfx_mlp_pack(int C, const float* w1, const float* b1, const float* w2, const float* b2, const float* gamma,
                 const float* beta, float* stream, float* params, int* workspace, void* stream_);
int sfx_block_mlp(int M, int C, const float* x, long long ldx, const float* stream, const float* params, float eps,
                  float* y, long long ldy, int* rowexp, void* stream_);
/* (ABI v13) rowexp (optional, [M] int32): also writes sfx_subm_rowexp(y) -- the next Block's fused SubM conv input
 * exponents -- from the output rows it just computed */
/* (ABI v13) training forward of the same tail (train.py:240-289, model.train()): also stores z [M][4C] (contiguous)
 * = fc1(LN2(x)), the pre-activation the backward needs, and applies the DropPath keep factor rowscale [M] (NULL:
 * none) to the branch: y = x + rowscale * (fc2(GELU(z)) + b2). */
int sfx_block_mlp_train(int M, int C, const float* x, long long ldx, const float* stream, const float* params,
                        float eps, const float* rowscale, float* z, float* y, long long ldy, void* stream_);
/* (ABI v13) its backward up to LN2: dh2 = W1^T (GELU'(z) o W2^T (rowscale * dy)), stream / params packed by
 * sfx_mlp_pack(C, W2^T [4C][C], zeros(4C), W1^T [C][4C], zeros(C), gamma, beta); LN2's backward + the residual are
 * the caller's (sfx_layernorm_bwd with dR = dy). */
int sfx_block_mlp_bwd(int M, int C, const float* dy, long long lddy, const float* stream, const float* params,
                      const float* rowscale, const float* z, float* dh2, long long lddh, void* stream_);

/* (ABI v11) Block.cpe + shortcut + norm1 in one launch (reference calflops.py:45-53: x1 = x + LN_cpe(Linear(
 * SubMConv3d(x))), h = norm1(x1); Pointcept Block.cpe = spconv SubMConv3d k=3 -> Linear -> LayerNorm), the
 * SubM pair products summed on chip (no per-pair partial rows, no atomics; rows' sums formed in ascending offset
 * order: bitwise reproducible).  C in {64, 96, 128}; rows contiguous [n][C], 16-byte aligned.
 * sfx_subm_cpe_pack (once per weight version): w = the CPE conv with the Linear folded in, W' [C][27 C]
 *   (row o, column k C + i: spconv [Cout, 3, 3, 3, Cin]) -> wpk (sfx_subm_cpe_pack_bytes(C) bytes of fp16x2
 *   fragments) + winv [C] (inverse column scales); ws: C floats.
 * sfx_subm_cpe_ln: xc = the conv input, xres = the shortcut (they differ for the first Block after an
 *   unpooling: Pointcept's stale sparse_conv_feat), nbr [n][27] (sfx_subm_neighbors), bias = the folded b'. */
size_t sfx_subm_cpe_pack_bytes(int C);
int sfx_subm_cpe_pack(int C, const float* w, void* wpk, float* winv, float* ws, void* stream);
int sfx_subm_cpe_ln(int n, int C, const float* xc, const float* xres, const int* nbr, const void* wpk,
                    const float* winv, const float* bias, const float* gamma_cpe, const float* beta_cpe,
                    const float* gamma1, const float* beta1, float eps, float* x_out, float* h_out, void* stream);

/* (ABI v11) PTv3 embedding (reference pointtransformer_v3.py:273-278: Linear(Cin, C) -> BatchNorm1d eval ->
 * GELU) on the VALU for Cin <= 64, C in {32, 64}: y[i] = GELU((x[i] W^T + b) * scale + shift); x rows strided
 * (ldx), y [n][ldy] 16-byte aligned; b / scale / shift may be NULL. */
int sfx_point_embed(int n, int K, int N, const float* x, long long ldx, const float* w, const float* b,
                    const float* scale, const float* shift, float* y, long long ldy, void* stream);

/* (ABI v11) FeaturePredictor output heads in one launch (reference models/feature_predictor.py:74-94, :201-235):
 * per head g (ng <= 6): Linear(kin, 128) -> ReLU -> Linear(128, 128) -> ReLU -> Linear(128, 128) -> ReLU ->
 * Linear(128, c_g); tanh on the first n_tanh output columns; + the residual record x[:, res_off:res_off+out_dim].
 * Hidden activations stay in registers (fp16x2 MFMA, fp32 accumulation; the last layer in fp32 on the VALU).
 * sfx_heads_pack (once per weight version): w1 [ng*128][ld1] (the six first layers concatenated, kin columns
 *   used), b1 [ng*128], wm [2][ng][128][128], bm [2][ng][128], w4 [out_dim][128] (each output row over its own
 *   head's units), b4 [out_dim] -> stream (sfx_heads_stream_floats) + params (sfx_heads_params_floats);
 *   ws: 3 ng 128 ints.
 * sfx_heads: x [M][ldx] (kin <= 160, 16-byte aligned rows), ocols[ng + 1] = head output column starts,
 *   y [M][out_dim] (out_dim <= 64). */
size_t sfx_heads_stream_floats(int ng, int kin);
size_t sfx_heads_params_floats(int out_dim);
int sfx_heads_pack(int ng, int kin, int out_dim, const float* w1, int ld1, const float* b1, const float* wm,
                   const float* bm, const float* w4, const float* b4, float* stream, float* params, int* ws,
                   void* stream_);
int sfx_heads(int M, int ng, int kin, int out_dim, const float* x, long long ldx, int res_off, int n_tanh,
              const int* ocols, const float* stream, const float* params, float* y, void* stream_);

#ifdef __cplusplus
}
#endif

#endif /* SFX_H_ */
