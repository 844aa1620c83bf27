/*
 * dgs.h — C ABI of libdgs_hip.so, the MI355X (gfx950) deformable-Gaussian training path.
 *
 * Plain pointers and sizes only: every float / int pointer is a DEVICE pointer (HBM) unless the comment
 * says "host"; every entry point enqueues on `stream` (a hipStream_t passed as void*) and returns
 * 0 on success or a negative dgs_status; dgs_last_error() gives the message.
 *
 * Reference interfaces replaced (preacherwhite/Deformable-3D-Gaussians):
 *   dgs_raster_forward   <- diff_gaussian_rasterization._C.rasterize_gaussians, called through
 *                           GaussianRasterizer.forward at gaussian_renderer/__init__.py:115-124
 *                           (submodule .gitmodules:4-7, un-vendored; contract: SURVEY.md section 8a R1-R9)
 *   dgs_raster_backward  <- diff_gaussian_rasterization._C.rasterize_gaussians_backward (autograd
 *                           of the same call; grads consumed at train_baseline.py:128,163-165)
 *   dgs_raster_ctx_free  <- release of the geometry/binning/image buffers the upstream op keeps in
 *                           its autograd ctx
 *   dgs_mark_visible     <- diff_gaussian_rasterization._C.mark_visible (GaussianRasterizer.markVisible)
 *   dgs_deform_*         <- DeformNetworkBaseline.forward / autograd backward
 *                           (utils/time_utils.py:56-127, called via scene/deform_model.py:323-324)
 *   dgs_knn_dist2        <- simple_knn._C.distCUDA2 (scene/gaussian_model.py:20,105-106)
 *   dgs_l1_ssim_*        <- l1_loss + ssim (utils/loss_utils.py:18-73) as used at train_baseline.py:126-127
 *   dgs_gaussian_inputs_* <- the glue of render() (gaussian_renderer/__init__.py:70-112: xyz + d_xyz,
 *                           exp(scaling) + d_scaling, normalize(rotation) + d_rotation, sigmoid(opacity),
 *                           cat(features_dc, features_rest)) and its autograd; *_se3_* and dgs_se3_*
 *                           the 6-DoF branch (gaussian_renderer/__init__.py:71-76, utils/rigid_utils.py)
 *   dgs_adam_step        <- torch.optim.Adam(..., eps=1e-15).step() of scene/gaussian_model.py:132 and
 *                           scene/deform_model.py:266 (train_baseline.py:176-182)
 */
#ifndef DGS_H
#define DGS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    DGS_OK = 0,
    DGS_ERR_ARGS = -1,      /* bad argument combination (upstream raises Exception) */
    DGS_ERR_HIP = -2,       /* a HIP runtime/launch error */
    DGS_ERR_UNSUPPORTED = -3,
    DGS_ERR_OOM = -4
} dgs_status;

/* GaussianRasterizationSettings (gaussian_renderer/__init__.py:53-66). The four tensor fields of
 * the reference (bg, viewmatrix, projmatrix, campos) are device pointers so no host sync is needed. */
typedef struct dgs_raster_settings {
    int image_height;
    int image_width;
    float tanfovx;
    float tanfovy;
    const float *bg;          /* (3,) device */
    float scale_modifier;
    const float *viewmatrix;  /* (4,4) device, world_view_transform (row-vector convention) */
    const float *projmatrix;  /* (4,4) device, full_proj_transform */
    int sh_degree;            /* active degree D (0..3) */
    const float *campos;      /* (3,) device */
    int prefiltered;
    int debug;                /* synchronise + check after every kernel */
} dgs_raster_settings;

typedef struct dgs_raster_ctx dgs_raster_ctx;

const char *dgs_last_error(void);
const char *dgs_version(void);

/* Forward. Exactly one of {shs, colors_precomp} and one of {(scales, rotations), cov3D_precomp}
 * must be non-NULL. P Gaussians, M SH coefficients per colour channel (shs is (P, M, 3)).
 * Outputs: out_color (3,H,W), out_depth (1,H,W), out_radii (P,) int32.
 * *ctx receives the saved state for dgs_raster_backward; *num_rendered (host) = tile pairs. */
int dgs_raster_forward(const dgs_raster_settings *s, int P, int M,
                       const float *means3D, const float *shs, const float *colors_precomp,
                       const float *opacities, const float *scales, const float *rotations,
                       const float *cov3D_precomp,
                       float *out_color, float *out_depth, int *out_radii,
                       dgs_raster_ctx **ctx, int *num_rendered, void *stream);

/* Backward. dL_ddepth may be NULL. Every output array is fully written (zeros where culled).
 * dL_dmeans2D / dL_dmeans2D_densify are (P,3) with z = 0 (NDC units, like upstream).
 * dL_dcolors is written only when forward got colors_precomp; dL_dcov3D only for cov3D_precomp;
 * dL_dshs / dL_dscales / dL_drotations only in the opposite cases (others may be NULL). */
int dgs_raster_backward(dgs_raster_ctx *ctx, const float *dL_dcolor, const float *dL_ddepth,
                        float *dL_dmeans3D, float *dL_dmeans2D, float *dL_dmeans2D_densify,
                        float *dL_dcolors, float *dL_dopacity, float *dL_dcov3D, float *dL_dshs,
                        float *dL_dscales, float *dL_drotations, void *stream);

/* Split-SH variant used by render()'s training path: the SH rows come straight from the Gaussian
 * model's features_dc (P,1,3) and features_rest (P,15,3) (scene/gaussian_model.py:71-74 concatenates
 * them per call; here the preprocess kernels read and write both tensors directly, so no (P,16,3)
 * copy is made either way). Degree <= 3, 16 coefficients; all four SH pointers 16-byte aligned.
 * Same outputs and semantics as dgs_raster_forward(shs = cat(features_dc, features_rest)); the
 * backward writes the two SH gradients. out_visible (P bytes, may be NULL) receives radii > 0, render()'s
 * visibility_filter (gaussian_renderer/__init__.py:130), from the preprocess kernel itself. */
int dgs_raster_forward_split_sh(const dgs_raster_settings *s, int P, const float *means3D,
                                const float *features_dc, const float *features_rest, const float *opacities,
                                const float *scales, const float *rotations, float *out_color, float *out_depth,
                                int *out_radii, uint8_t *out_visible, dgs_raster_ctx **ctx, int *num_rendered,
                                void *stream);
int dgs_raster_backward_split_sh(dgs_raster_ctx *ctx, const float *dL_dcolor, const float *dL_ddepth,
                                 float *dL_dmeans3D, float *dL_dmeans2D, float *dL_dmeans2D_densify,
                                 float *dL_dopacity, float *dL_dfeatures_dc, float *dL_dfeatures_rest,
                                 float *dL_dscales, float *dL_drotations, void *stream);

void dgs_raster_ctx_free(dgs_raster_ctx *ctx);
/* The pair count of ctx's forward (resolving a deferred count: a host wait for the GPU's read-back);
 * the count the binning used, i.e. the speculative capacity if it overflowed. -1 on error. */
int dgs_raster_ctx_num_rendered(dgs_raster_ctx *ctx);

/* Frustum test only (p_view.z > 0.2): visible (P,) uint8. */
int dgs_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *visible, void *stream);

/* ---- binning debug hooks (tests only) ----
 * The forward launches tile binning for a learned per-device pair capacity before it knows the
 * pair count (speculative binning) and redoes binning at the exact size when the count is larger.
 * dgs_debug_set_pair_cap overrides that capacity for `device` (0 = none: the next forward runs
 * synchronously); dgs_debug_pair_cap reads it back; dgs_debug_binning_redos counts the redone
 * (overflowing) launches so far. dgs_debug_set_binning selects the binning: 0 = rect binning
 * (count -> column scan -> place; the default where its LDS bound allows), 1 = duplicate + tile-key
 * radix sort + ranges (the scheme of the external upstream rasterizer's duplicateWithKeys / SortPairs /
 * identifyTileRanges, SURVEY.md section 3 kernel table). */
/* Deferred pair count (training steps that can be redone): with it on, a speculative forward
 * returns without waiting for num_rendered (*num_rendered = -1); the backward (or ctx_free) reads
 * it. If it exceeded the speculative capacity the forward's image was computed on truncated tile
 * lists: dgs_raster_deferred_overflows() counts these, and the caller must redo the step with the
 * mode off (deformgs/train_step.py does). The backward of such a step stays in bounds. Off by
 * default (the upstream op's synchronous num_rendered). */
void dgs_raster_set_deferred_count(int on);
long long dgs_raster_deferred_overflows(void);
void dgs_debug_set_pair_cap(int device, int cap);
int dgs_debug_pair_cap(int device);
void dgs_debug_set_binning(int mode);
long long dgs_debug_binning_redos(void);
/* Blend backward scheme (rect binning, no depth gradient): 1 = segmented (k_blend_bwd2s: every 128 list
 * positions of a tile an independent work item, started from per-pixel checkpoints the forward writes);
 * 0 = one serial back-to-front replay per tile (k_blend_bwd2). Default from DGS_BLEND_SEG. Applies to
 * forwards issued after the call. */
void dgs_debug_set_blend_seg(int on);
/* The blend-backward mode in effect (DGS_BLEND_SEG or the last dgs_debug_set_blend_seg): 1 = segmented. */
int dgs_debug_get_blend_seg(void);
/* Deterministic blend backward (rect binning): 1 = every (tile, Gaussian) pair's gradient terms are written
 * to per-pair slots and summed per Gaussian in a fixed order (k_rect_gather) instead of float atomics, so
 * repeated backwards of the same forward give bitwise-identical gradients (the upstream renderCUDA backward's
 * global atomics, SURVEY.md §2 renderCUDA row and §7 risk (c), are order-dependent). Costs the slot traffic; off by
 * default (DGS_DETERMINISTIC=1 turns it on). Applies to backwards issued after the call. */
void dgs_raster_set_deterministic(int on);
int dgs_raster_get_deterministic(void);
/* Rect binning order: 1 (default; DGS_TILE_SORT=0 turns it off) = the Gaussians are binned in index order
 * and each tile's list is then sorted by (depth, index) in its own workgroup (k_tile_sort); 0 = a global
 * stable depth sort first (4 radix passes), lists placed in that order. The lists are identical either
 * way. The deterministic backward keeps the per-tile sort: k_tile_sort also writes each sorted entry's
 * index-order position, where the backward stores the pair's sums for k_rect_gather. Applies to forwards
 * issued after the call. */
void dgs_debug_set_tile_sort(int on);
int dgs_debug_get_tile_sort(void);
/* Forward blend with two pixels per lane (k_blend_fwd2; DGS_BLEND_FWD2=1): 1 = on. Images, transmittance and
 * per-pixel contributor counts are bitwise those of the default k_blend_fwd. Applies to forwards issued
 * after the call (not with the segmented backward's checkpoints). */
void dgs_debug_set_blend_fwd2(int on);
int dgs_debug_get_blend_fwd2(void);
/* host nanoseconds spent waiting for num_rendered (and the number of waits) since process start */
long long dgs_debug_count_wait_ns(long long *waits);
/* dL/dscales convention. 0 (default) = the upstream CUDA op's: the gradient w.r.t. the modified scale
 * scale_modifier * s (its computeCov3D backward omits the factor); 1 = the chain rule through the
 * modifier (dL/ds). Identical when scale_modifier == 1 (every training call: render() default). */
void dgs_raster_set_exact_scale_grad(int on);
/* Times the deformation MLP's barrier-free LDS hand-off gave up waiting (bounded spin expired) on the
 * current device since process start: must be 0; a non-zero count means MLP outputs / gradients of
 * some launch are invalid (GPU tests assert it stays 0). -1 if the counter could not be read. */
long long dgs_debug_guard_expiries(void);
/* dW launches of the split-f16 path handed to the fp32 k_dw since process start: a 256-row dZ / saved
 * operand spans >= 2^31 bytes (N > ~2.1 M points), past k_dws's 32-bit buffer offsets (the fp32 k_dw
 * takes up to ~8.4 M). Same results to fp32 summation order (tests/test_gpu_mlp.py linearity test). */
long long dgs_debug_dw_fallbacks(void);
/* CUs the deformation-MLP kernels leave free for concurrent work on other streams (the data-parallel
 * step's gradient all-reduce under the network backward): the persistent k_fwd / k_bwd
 * grids launch (CUs - k) workgroups and k_dws's plan spans (256 - k). 0..64; default
 * DGS_MLP_RESERVE_CUS or 0. No reference counterpart (the reference is single-GPU). */
void dgs_mlp_set_reserved_cus(int k);
int dgs_mlp_reserved_cus(void);
/* Diagnostic: a stand-in for an RCCL ring all-reduce on `stream` (nwg workgroups of 256 threads,
 * `passes` read-modify-write sweeps over n floats of a 16-byte aligned buffer; values unchanged up to
 * rounding), for measuring on one GPU whether a collective overlaps the network backward
 * (tools/overlap_probe.py). */
int dgs_debug_collective_standin(float *buf, long long n, int nwg, int passes, void *stream);
/* The binning's stable LSD radix sort on device buffers (tests only): sorts n (key, value) pairs by
 * key bits [0, end_bit) (32-bit keys when key_bytes == 4, 16-bit when 2; end_bit <= 8 * key_bytes)
 * using (k1, v1) as scratch; the result is left in (k0, v0). Stream-ordered. */
int dgs_debug_sort_pairs(void *k0, void *k1, uint32_t *v0, uint32_t *v1, int n, int key_bytes, int end_bit,
                         void *stream);

/* ---- timing hooks (bench.py): per-kernel-class HIP event accumulation on the launch stream ---- */
void dgs_timing_enable(int on);
/* Restrict timing to the comma-separated kernel classes in `csv` (host string; NULL or "" = all). */
void dgs_timing_select(const char *csv);
/* Returns accumulated ms for kernel class `name` and its launch count (host); syncs those events. */
double dgs_timing_query(const char *name, int *launches);
void dgs_timing_reset(void);
/* Time only every `period`-th launch of each selected class (1 = every launch, the default): each
 * timed launch costs two stream markers, ~6 us of GPU idle each. */
void dgs_timing_sample(int period);
/* Launches of a selected class since the last reset, timed or not (timed = ceil(launches / period)). */
long long dgs_timing_launches(const char *name);

/* ---- deformation MLP (utils/time_utils.py:56-201), fused PE + 8x256 MLP ----
 * Default: fp32 GEMMs on f16 MFMA over a scaled two-piece operand split (x * 2^e = hi + lo, both f16;
 * three products hh + hl + lh per fp32 product, dropped ll <= 2^-22 relative; every output and
 * gradient held to 2x the fp32-MFMA path's error, mlp_split.hip). DGS_MLP_EXACT_FP32 selects the
 * v_mfma_f32_32x32x2_f32 kernels (bit-identical to fp32 fma chains). The flag changes the packed /
 * saved / scratch layouts: pass the same flags to every call of one forward/backward. */
enum {
    DGS_MLP_BLENDER = 1,   /* timenet on (t: L=6 -> 256 -> 30); else raw t PE (L=10, 21 ch) */
    DGS_MLP_6DOF = 2,      /* heads branch_w(3), branch_v(3) instead of gaussian_warp(3) */
    DGS_MLP_NO_ROTSCALE = 4, /* DeformNetwork fork variant: rotation/scaling heads unused */
    DGS_MLP_EXACT_FP32 = 8, /* fp32-input MFMA path instead of the split-f16 path */
    DGS_MLP_UNIFORM_T = 16  /* caller guarantees t[i] == t[0] for every point (one frame time, as
                               train_baseline.py:107-110 feeds it): the timenet runs once per launch,
                               t_emb is folded into the linear.0 / linear.5 biases (outputs equal the
                               per-point path to fp32 rounding), and the timenet / t_emb-column
                               gradients are formed from the layer-0/5 bias gradients instead of
                               per-point sums (split path, blender only; ignored otherwise) */
};

/* Parameter table: device pointers in state_dict order of DeformNetworkBaseline
 * (timenet.0.w, timenet.0.b, timenet.2.w, timenet.2.b [blender only], linear.0.w, linear.0.b, ...,
 *  linear.7.b, then head weights/biases: warp|branch_w[,branch_v], rotation, scaling). */
int dgs_deform_num_params(int flags);
size_t dgs_deform_packed_floats(int flags);
/* floats of activation storage kept by forward for backward (N points) */
size_t dgs_deform_saved_floats(int flags, int N);
size_t dgs_deform_scratch_floats(int flags, int N);
int dgs_deform_pack(int flags, const float *const *params, float *packed, void *stream);
/* out: (N, n_out) with n_out = 10 (d_xyz3, d_rot4, d_scale3) or 13 for 6-DoF (w3, v3, rot4, scale3).
 * t: (N,1) per-point time. saved may be NULL for inference (no backward). */
int dgs_deform_forward(int flags, int N, const float *xyz, const float *t, const float *packed,
                       float *out, float *saved, void *stream);
/* dgs_deform_pack + dgs_deform_forward in one call (the training step's order): the same launches as the
 * two calls (pack, then k_timenet and the forward), results bitwise equal. */
int dgs_deform_pack_forward(int flags, const float *const *params, int N, const float *xyz, const float *t,
                            float *packed, float *out, float *saved, void *stream);
/* dout: (N, n_out). grads: device pointers in the same order as params (overwritten).
 * scratch: dgs_deform_scratch_floats(flags, N) floats. */
int dgs_deform_backward(int flags, int N, const float *packed, const float *saved, const float *dout,
                        float *scratch, float *const *grads, void *stream);
int dgs_deform_outputs(int flags);

/* ---- fused photometric loss (utils/loss_utils.py:18-73, train_baseline.py:126-127) ----
 * img, gt: (C,H,W). out3 (device) = [loss, mean L1, mean SSIM] with
 * loss = (1-lambda) * L1 + lambda * (1 - SSIM). scratch: dgs_l1_ssim_scratch_floats floats, kept
 * from forward for backward. dloss (device scalar, may be NULL = 1) scales dL/dimg. */
size_t dgs_l1_ssim_scratch_floats(int C, int H, int W);
int dgs_l1_ssim_forward(int C, int H, int W, const float *img, const float *gt, float lambda, float *out3,
                        float *scratch, void *stream);
int dgs_l1_ssim_backward(int C, int H, int W, const float *img, const float *gt, float lambda,
                         const float *scratch, const float *dloss, float *grad, void *stream);
/* The 11 separable window taps the loss kernels filter with (host-side, no GPU): the reference's 1-D
 * Gaussian with its outer product's total matched to the reference's fp32 2-D window (ssim.hip). */
void dgs_l1_ssim_window(float *out11);

/* ---- simple-knn replacement: mean squared distance to the 3 nearest neighbours ---- */
int dgs_knn_dist2(int P, const float *points, float *dist2, void *stream);

/* ---- rasterizer inputs of render() (gaussian_renderer/__init__.py:70-112, gaussian_model.py:39-50) ----
 * means3D = xyz + d_xyz; scales = exp(scaling) + d_scaling; rotations = normalize(rotation) + d_rotation;
 * opacities = sigmoid(opacity); shs (P, 1 + M_rest, 3) = cat(features_dc (P,1,3), features_rest (P,M_rest,3)).
 * deform: rows of deform_stride floats holding [d_xyz(3) d_rotation(4) d_scaling(3)] (the deformation
 * network output), or NULL for no deformation. Backward: g_* outputs may be NULL (not needed);
 * g_deform receives the same row layout. shs == NULL (forward) / d_shs == NULL (backward): the SH
 * rows are not concatenated / split (dgs_raster_*_split_sh reads and writes them in place). */
int dgs_gaussian_inputs_forward(int P, int M_rest, const float *xyz, const float *f_dc, const float *f_rest,
                                const float *scaling, const float *rotation, const float *opacity,
                                const float *deform, int deform_stride, float *means3D, float *shs,
                                float *scales, float *rotations, float *opacities, void *stream);
int dgs_gaussian_inputs_backward(int P, int M_rest, const float *scaling, const float *rotation,
                                 const float *opacity, const float *d_means3D, const float *d_shs,
                                 const float *d_scales, const float *d_rotations, const float *d_opacities,
                                 float *g_xyz, float *g_dc, float *g_rest, float *g_scaling, float *g_rotation,
                                 float *g_opacity, float *g_deform, int deform_stride, void *stream);
/* 6-DoF variant (render(..., is_6dof=True), gaussian_renderer/__init__.py:71-76 with the screw head of
 * utils/time_utils.py:114-121 and exp_se3 of utils/rigid_utils.py:4-83 in the same launch): deform rows
 * (deform_stride >= 13, required) hold [w_r(3) v_r(3) d_rotation(4) d_scaling(3)], the raw head
 * outputs; theta = |w_r|, w = w_r/theta + 1e-5, v = v_r/theta + 1e-5, (R, p) = exp_se3(w, v, theta),
 * means3D = R xyz + p. Backward also needs xyz and the deform rows; g_deform uses deform_stride. */
int dgs_gaussian_inputs_se3_forward(int P, int M_rest, const float *xyz, const float *f_dc, const float *f_rest,
                                    const float *scaling, const float *rotation, const float *opacity,
                                    const float *deform, int deform_stride, float *means3D, float *shs,
                                    float *scales, float *rotations, float *opacities, void *stream);
int dgs_gaussian_inputs_se3_backward(int P, int M_rest, const float *xyz, const float *deform, int deform_stride,
                                     const float *scaling, const float *rotation, const float *opacity,
                                     const float *d_means3D, const float *d_shs, const float *d_scales,
                                     const float *d_rotations, const float *d_opacities, float *g_xyz, float *g_dc,
                                     float *g_rest, float *g_scaling, float *g_rotation, float *g_opacity,
                                     float *g_deform, void *stream);
/* exp_se3 of the raw screw head -> M (P, 4, 4) = rp_to_se3(R, p) (the d_xyz DeformNetwork returns for
 * is_6dof, utils/time_utils.py:114-121 / utils/rigid_utils.py:27-35), and its backward: dM (P, 4, 4)
 * -> g_raw columns 0..5 (rows of g_stride floats); M's constant last row passes no gradient. */
int dgs_se3_forward(int P, const float *raw, int raw_stride, float *M, void *stream);
int dgs_se3_backward(int P, const float *raw, int raw_stride, const float *dM, float *g_raw, int g_stride,
                     void *stream);

/* ---- Adam over many tensors in one launch (torch.optim.Adam, amsgrad/weight_decay off) ----
 * Per tensor (host array of n descriptors, device data pointers):
 *   m = lerp(m, g, 1 - beta1); v = beta2 v + (1 - beta2) g^2;
 *   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps)
 * with step_size = lr / (1 - beta1^t) and bc2_sqrt = sqrt(1 - beta2^t) computed by the caller;
 * 1 - beta1 and 1 - beta2 are formed in double and rounded to float (torch's scalar handling). */
typedef struct dgs_adam_tensor {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t numel;
    float step_size;
    float bc2_sqrt;
} dgs_adam_tensor;
int dgs_adam_step(int n, const dgs_adam_tensor *tensors, double beta1, double beta2, double eps, void *stream);

/* ---- Row selection (stream compaction) over many tensors in one launch ----
 * Replaces the per-tensor boolean indexing of densification: prune_points / _prune_optimizer
 * (t[mask] for every parameter, both Adam moments and the statistics) and the row gathers of
 * densify_and_clone / densify_and_split (scene/gaussian_model.py:206-246, 280-312 upstream
 * layout). For every job, dst[k] = src[i] for the k-th row i (in order) with mask[i] != 0; rows are
 * `width` contiguous floats, dst holds sum(mask != 0) rows. mask: nrows bytes (0 / 1, device). */
typedef struct dgs_row_job {
    const float *src;
    float *dst;
    int width;
} dgs_row_job;
int dgs_select_rows(int nrows, const uint8_t *mask, int njobs, const dgs_row_job *jobs, void *stream);

/* ---- one training iteration in one call (train_baseline.py:104-128) ----
 * deform.step -> render() input glue -> split-SH rasterizer -> (1 - lambda) L1 + lambda (1 - SSIM) ->
 * backward (loss, rasterizer, input glue, deformation network): the fused path of
 * deformgs/train_step.forward_backward issued from C++ (same entry points, same order, same stream)
 * instead of through the PyTorch autograd engine. All buffers are the caller's, sized for P; gradients
 * are overwritten in place (dgs_adam_step reads them). deform = 0: the warm-up iterations (deltas 0.0,
 * the network does not run; train_baseline.py:106-107). t: device scalar, the frame time fid +
 * ast_noise (train_baseline.py:107-112); t_full (P floats) is needed unless the network is the blender
 * one on the split path (whose kernels read t[0]). deferred_count: as dgs_raster_set_deferred_count for
 * this call; *overflowed = 1 when the speculative pair capacity overflowed (redo the step with 0).
 * *num_rendered = the pair count (a deferred count is resolved at the end of the call).
 * phase (data-parallel steps, deformgs/native_step.py): bit 1 = everything up to the Gaussian parameter
 * gradients (the network's dL/d(output) included), the pair count resolved at its end; bit 2 = the
 * network backward (dX, dW) of the preceding bit-1 call; 0 = both (one call). Between the two the
 * caller agrees on an overflow redo and starts the Gaussian gradient all-reduce, which then overlaps
 * the network backward. */
typedef struct dgs_train_step_args {
    int P;
    const float *xyz, *f_dc, *f_rest, *scaling, *rotation, *opacity;   /* (P,3) (P,1,3) (P,15,3) (P,3) (P,4) (P,1) */
    int deform;
    int mlp_flags;                       /* DGS_MLP_* of the network (DGS_MLP_UNIFORM_T is implied) */
    const float *const *mlp_params;      /* host array of device pointers, dgs_deform_pack order */
    float *const *mlp_grads;             /* host array, same order (overwritten) */
    float *mlp_packed, *mlp_saved, *mlp_scratch;  /* dgs_deform_{packed,saved,scratch}_floats */
    float *mlp_out, *mlp_dout;           /* (P, dgs_deform_outputs) */
    const float *t;
    float *t_full;
    dgs_raster_settings rs;
    const float *gt;                     /* (3,H,W) */
    float lambda_dssim;
    float *means3D, *scales, *rotations, *opacities;  /* render inputs (P,3) (P,3) (P,4) (P,1) */
    float *image, *depth;                /* (3,H,W) (1,H,W) */
    int *radii;                          /* (P,) */
    uint8_t *visible;                    /* (P,) radii > 0, may be NULL */
    float *loss3, *loss_scratch, *dimage;   /* (3,): loss, L1, SSIM; dgs_l1_ssim_scratch_floats; (3,H,W) */
    float *d_means3D, *d_means2D, *d_means2D_densify, *d_opacities, *d_scales, *d_rotations;
    float *g_xyz, *g_dc, *g_rest, *g_scaling, *g_rotation, *g_opacity;  /* parameter gradients */
    int deferred_count;
    int phase;                           /* 0 (= 3), 1, 2, 3: see above */
} dgs_train_step_args;
int dgs_train_step(const dgs_train_step_args *a, int *overflowed, int *num_rendered, void *stream);

#ifdef __cplusplus
}
#endif
#endif
