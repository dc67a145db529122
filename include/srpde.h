/*
 * srpde.h -- C ABI of libsrpde_hip.so, the MI355X (gfx950) kernels behind the
 * superresolution_for_pdes_amd drop-in for tahmidawal/Superresolution_for_PDEs.
 *
 * The reference is pure Python (no FFI layer); its hot path dispatches PyTorch aten ops
 * from src/models.py and SciPy's SuperLU from src/data_generation.py.  Each entry point
 * below replaces the aten / SciPy call(s) cited next to it.  The Python binding is
 * superresolution_for_pdes_amd/_lib.py (ctypes); INTEGRATION.md shows the stub a
 * maintainer would add on the reference side.
 *
 * Conventions
 *  - All tensor arguments are caller-owned DEVICE pointers; the library never allocates,
 *    frees or synchronises the host (one exception: srpde_poisson_cg_batched for a single problem
 *    too large for one cooperative grid, n > 1024).  Scratch is passed in as (workspace, ws_bytes), its
 *    size queried with the matching *_workspace_size() function.
 *  - Activations are NHWC fp32 ("channels-last").  A view is (pointer, ld): ld = floats
 *    between consecutive pixels, so channel slices of a wider tensor (virtual concat) need
 *    no copy.  Channel counts and ld must be multiples of 4; pointers 16-byte aligned.
 *  - Every call is stream-ordered on `stream` (on ROCm torch.cuda.current_stream().cuda_stream).
 *  - The library holds no global mutable state and reads no environment: every choice (kernel family,
 *    test hooks) is an argument of the call, so calls are re-entrant from any thread.  (The one piece of
 *    per-thread state is diagnostic: srpde_last_error / srpde_last_kernel.)
 *  - Return: 0 on success, negative on a bad argument (-1 arg, -2 shape, -3 alignment,
 *    -4 workspace too small), positive hipError_t on a launch failure.  srpde_last_error()
 *    returns the thread-local message of the last failure.
 */
#ifndef SRPDE_H_
#define SRPDE_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;

/* ABI version: bumped whenever an exported signature or a documented buffer layout changes.
 * A binding built against this header checks srpde_version() == SRPDE_ABI_VERSION at load time
 *  and refuses a mismatched library instead of misreading arguments.
 *   1  round 1-2 layout
 *   4  round 3 changes (srpde_conv_fwd_h3: in_scale ... ep_amax before the workspace; the
 *      srpde_prepare_weights_h3 descriptor row grew to 10 columns; srpde_conv_wgrad_h3p reads dy
 *      planes with a row stride of cout rounded up to 32) and round 4's additions
 *      (srpde_conv_h4_set, srpde_poisson_debug_abort)
 *   5  srpde_conv_fwd_h3: x1_ca, x1_sa before the workspace
 *   6  srpde_conv_fwd: ep_mean, ep_invstd, ep_gamma, ep_beta, ep_amax before the workspace
 *   7  srpde_conv_fwd_h3: x0_up, up_ld, up_h, up_w before the workspace; srpde_upsample_gate_sa;
 *      srpde_conv_head_eval
 *   8  srpde_conv_h3_stats_rows_for, srpde_conv_h5_set (the h5 forward writes 80-row statistics),
 *      srpde_conv_head_eval_supported, srpde_last_kernel
 *   9  srpde_conv_wgrad_h3x, srpde_conv_wgrad_h3x_supported, srpde_bn_train_finalize_ws,
 *      srpde_bn_finalize_workspace_size
 *  10  no global state: srpde_conv_h5_set / _h4_set / _h3r_set and srpde_poisson_debug_abort removed; the kernel
 *      family is SRPDE_FAM_* bits of srpde_conv_fwd_h3's / _presplit's accumulate argument and of
 *      srpde_conv_h3_stats_rows_for's new flags argument, the grid-CG abort hook a negative rtol;
 *      srpde_conv_wgrad_h3g_supported, srpde_att_pool_bn_bwd(_blocks); srpde_att_bwd takes dx == NULL
 *  11  srpde_upsample_bilinear_bwd_gated_bn, srpde_upsample_bwd_bn_supported, srpde_gating_bn_reduce(_blocks),
 *      srpde_att_bwd_params_lowres, srpde_conv_wgrad_bnb */
#define SRPDE_ABI_VERSION 11

/* Kernel-family bits (per call; bit 0 of the same argument is the accumulate flag): the forward / dgrad
 * families compute the same outputs, statistics and stored splits bit for bit, so these only route a call to
 * another kernel -- tests compare the families, tuning times them.  SRPDE_FAM_NO_H5: not the W = 40 h5 kernel
 * (nor out_conv2's 16-output kernel); SRPDE_FAM_NO_H4: not the h4 one-tap-ring kernel (W = 10 / 20 / 40 tiles);
 * SRPDE_FAM_NO_H3R: not the 4-wave, two-workgroups-per-CU kernel for <= 64-channel tiles. */
#define SRPDE_FAM_NO_H5 2
#define SRPDE_FAM_NO_H4 4
#define SRPDE_FAM_NO_H3R 8

const char* srpde_last_error(void);
/* Name of the main kernel the last conv entry point (srpde_conv_fwd*, srpde_conv_dgrad_h3_bnb, srpde_conv_wgrad*,
 * srpde_conv_head_eval) launched on this thread, as profilers print it, e.g. "conv_fwd_h5_kernel<2, 8>" (template
 * arguments included, namespace and parameter list dropped).  Diagnostics / per-kernel roofline accounting. */
const char* srpde_last_kernel(void);
int srpde_version(void);

/* ---- convolution: nn.Conv2d 3x3 (dilation 1|2) / 1x1 -------------------------------
 * replaces aten::convolution (fwd) and aten::convolution_backward (dgrad, wgrad) for
 * ConvBlock.conv1/conv2 (src/models.py:16,18,22-23), bridge[0]/[3] (models.py:43,46),
 * out_conv1/out_conv2 (models.py:57,59).  torch.cat (models.py:87,90,93) is absorbed as
 * the (x1, c1) second input.  stats (nullable): per row-block (mean, M2) float2
 * partials for the train-mode BatchNorm that follows; srpde_conv_stats_blocks() blocks
 * of srpde_conv_stats_rows_per_block() rows each. */
int srpde_pack_conv_weights(const float* w, float* wfwd, float* wdgrad, int cout, int cin, int cin_real,
                            int ksize, hipStream_t stream);
int srpde_conv_fwd(const float* x0, int c0, int ldx0, const float* x1, int c1, int ldx1, const float* wpack,
                   const float* bias, float* y, int ldy, int n, int h, int w, int cout, int ksize, int dil,
                   int sign, int accumulate, float* stats, const float* ep_mean, const float* ep_invstd,
                   const float* ep_gamma, const float* ep_beta, unsigned* ep_amax, void* workspace,
                   size_t ws_bytes, hipStream_t stream);
/* ep_* (nullable, eval mode, layers with cin % 32 != 0 -- enc1.conv1): the epilogue applies the
 * following BatchNorm (running statistics) + ReLU, as srpde_conv_fwd_h3's ep_* below. */
/* optional scratch for splitting the last, partially filled round of tiles over K (pass
 * NULL to disable); srpde_conv_fwd_workspace_size() bytes always suffice */
size_t srpde_conv_fwd_workspace_size(int cout);
size_t srpde_conv_stats_blocks(int n, int h, int w, int cout);
int srpde_conv_stats_rows_per_block(int cout);
size_t srpde_conv_wgrad_workspace_size(int n, int h, int w, int cout, int cin, int ksize);
int srpde_conv_wgrad(const float* dy, int lddy, const float* x0, int c0, int ldx0, const float* x1, int c1,
                     int ldx1, float* dw, int cin_real, int accumulate, int n, int h, int w, int cout, int ksize,
                     int dil, void* workspace, size_t ws_bytes, hipStream_t stream);
/* srpde_conv_wgrad (fp32 kernels, one input) whose dY is the BN (+ReLU, flags SRPDE_BN_RELU) backward of the
 * layer's BatchNorm, applied as the operand is loaded: dy = gamma invstd (dz - m1 - xhat m2), dz = da masked by
 * the BN output > 0, y the BN input -- srpde_bn_relu_bwd's dy bit for bit from srpde_bn_bwd_prepare's m1 / m2,
 * never written (enc1.conv1, models.py:16-23 with the input image: no dgrad reads dy). */
int srpde_conv_wgrad_bnb(const float* da, int ldda, const float* y, int ldy, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, const float* m1, const float* m2, int flags,
                         const float* x0, int c0, int ldx0, float* dw, int cin_real, int accumulate, int n, int h,
                         int w, int cout, int ksize, int dil, void* workspace, size_t ws_bytes, hipStream_t stream);
/* h3: the same convolution (forward / dgrad, same output and statistics layout) from
 * two-piece fp16 splits with power-of-two operand scales: three partial products per fp32
 * product on v_mfma_f32_32x32x16_f16, halo-staged activation tiles (conv_h3.hip).
 * amax0/amax1: device words holding max|x0| / max|x1| as float bits (any upper bound within a
 * few orders of magnitude works; srpde_absmax or the amax output of srpde_bn_relu_fwd/_bwd).
 * wsplit/wexp: srpde_split_weights_h3 of the packed weights ([2][rows][K] fp16, [rows] int).
 * xsplit_out (nullable): receives the scaled hi / lo fp16 pieces of the input, [2][P][c0+c1],
 * for srpde_conv_wgrad_h3p (the split is computed anyway; storing it costs one 4-B write per
 * element). */
int srpde_conv_h3_supported(int c0, int c1, int cout, int w, int dil, int ksize);
/* Rows per BatchNorm-statistics block written by srpde_conv_fwd_h3 (stats / bn_part buffers
 * hold ceil(P / rows) blocks); the other conv families use srpde_conv_stats_rows_per_block. */
int srpde_conv_h3_stats_rows(void);
/* Rows per BatchNorm-statistics block srpde_conv_fwd_h3 writes for the FORWARD of this shape (input
 * channels c0 + c1 -> cout at h x w, dilation dil) and kernel-family bits `flags` (those the forward call
 * will pass): 80 where the h5 kernel takes it (w = 40, h % 8 == 0, cout 64 or 32, c0 + c1 a multiple of 64,
 * no SRPDE_FAM_NO_H5), else srpde_conv_h3_stats_rows().  Dgrad partials (bn_part) keep
 * srpde_conv_h3_stats_rows(). */
int srpde_conv_h3_stats_rows_for(int c0, int c1, int cout, int h, int w, int dil, int flags);
int srpde_split_weights_h3(const float* w, void* planes, int* wexp, int rows, int K, hipStream_t stream);
int srpde_absmax(const float* x, int ldx, int c, long long P, unsigned* amax, hipStream_t stream);
/* every conv layer's forward and dgrad h3 planes in one launch from torch's [Cout][Cin][3][3]
 * weights: desc = device int64 [nlayers][10] = {w, cout, cin_real, cin_pad, planes_f, exp_f,
 * planes_d, exp_d, first row, cout_pad}; a layer owns cout forward rows then cin_pad dgrad rows of
 * K = 9 * cout_pad (k = tap * cout_pad + n, zero for n >= cout) */
int srpde_prepare_weights_h3(const long long* desc, int nlayers, int total_rows, hipStream_t stream);
/* dgrad (conv^T) with the BatchNorm (+ReLU) backward apply of the layer fused into the operand
 * transform: dy = gamma*invstd*(dz - m1 - xhat*m2) is formed per halo element from da (the BN
 * output gradient) and bn_y_in (the BN input), never stored in fp32; m1, m2 and the dy scale bound
 * from srpde_bn_bwd_prepare.  dysplit_out [2][P][cout_dy] fp16: dy's split for
 * srpde_conv_wgrad_h3p.  bn_* / bn_part (nullable): the next BN's backward reduction as in
 * srpde_conv_fwd_h3; dx_max (nullable): per output tile max|dx| (ceil(P/256)*ceil(cin_dx/BN)
 * slots) for the next srpde_bn_bwd_prepare.  Replaces srpde_bn_relu_bwd + srpde_conv_fwd_h3(sign -1). */
int srpde_conv_h3_bnb_supported(int cout_dy, int cin_dx, int w, int dil);
int srpde_conv_dgrad_h3_bnb(const float* da, int ldda, const unsigned* dy_amax, const float* bn_y_in, int bn_ldy_in,
                            const float* mean, const float* invstd, const float* gamma, const float* beta,
                            const float* m1, const float* m2, int flags, const void* wsplit, const int* wexp,
                            float* dx, int lddx, int n, int h, int w, int cout_dy, int cin_dx, int dil,
                            void* dysplit_out, const float* bn_y, int bn_ldy, const float* bn_mean,
                            const float* bn_invstd, const float* bn_gamma, const float* bn_beta, void* bn_part,
                            float* dx_max, void* workspace, size_t ws_bytes, hipStream_t stream);
/* srpde_conv_fwd_h3 (no virtual concat, no input transform) on an input that arrives as its h3
 * split: xsplit = [2][P][c] fp16 hi / lo planes of x * 2^h3_exp(*amax) (srpde_bn_bwd_apply_split,
 * or a stored xsplit_out).  The halo tiles go into the MFMA operand layout as fp16 pieces (no fp32
 * tile, no split work, nothing stored for the weight gradient, which reads the same planes); same
 * outputs, statistics, bn_part and out_max as srpde_conv_fwd_h3 on that split. */
int srpde_conv_fwd_h3_presplit(const void* xsplit, int c, const unsigned* amax, const void* wsplit, const int* wexp,
                               const float* bias, float* y, int ldy, int n, int h, int w, int cout, int ksize,
                               int dil, int sign, int accumulate, float* stats, const float* bn_y, int bn_ldy,
                               const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                               const float* bn_beta, void* bn_part, float* out_max, void* workspace, size_t ws_bytes,
                               hipStream_t stream);
/* Output tiles (= out_max slots) of srpde_conv_fwd_h3 for P rows, cin -> cout; 0 if unsupported. */
long long srpde_conv_h3_tiles(long long P, int cin, int cout, int w, int dil);
int srpde_conv_fwd_h3(const float* x0, int c0, int ldx0, const float* x1, int c1, int ldx1, const unsigned* amax0,
                      const unsigned* amax1, const void* wsplit, const int* wexp, const float* bias, float* y, int ldy,
                      int n, int h, int w, int cout, int ksize, int dil, int sign, int accumulate, float* stats,
                      void* xsplit_out, const float* in_scale, const float* in_shift, const float* bn_y,
                      int bn_ldy, const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                      const float* bn_beta, void* bn_part, float* out_max, const float* ep_mean,
                      const float* ep_invstd, const float* ep_gamma, const float* ep_beta, unsigned* ep_amax,
                      const float* x1_ca, const float* x1_sa, const float* x0_up, int up_ld, int up_h, int up_w,
                      void* workspace, size_t ws_bytes, hipStream_t stream);
/* accumulate: bit 0 = y += conv; the SRPDE_FAM_* bits route the call away from a kernel family (tests /
 * tuning: the families' outputs are equal bit for bit); srpde_conv_fwd_h3_presplit reads it the same way. */
/* x1_ca [n][c1] / x1_sa [P] (nullable, together, c1 > 0): the second input is an AttentionGate's
 * input x (models.py:119-130) and the conv reads its gated output (x * ca[sample][c]) * sa[pixel]
 * (srpde_att_apply_fwd's expression, formed in the operand transform; xsplit_out and the statistics
 * are those of the gated input) -- the gated tensor is never written.
 * x0_up (nullable; up_ld its row stride, up_h = h / 2, up_w = w / 2): x0 is the bilinear x2
 * (align_corners) upsample of this [n][up_h][up_w][c0] tensor, formed in the operand transform from
 * its low-res rows (models.py:70, 89, 92: the decoder's upsampled input is never written); bit-identical
 * to reading srpde_upsample_bilinear_fwd's output.  Forward only, no in_scale, and the h4 shapes
 * (W 20 with 128-column tiles, W 40 with 64); x0 / ldx0 are ignored for the x0 channels; amax0 must
 * bound |up(x0_up)| (the source's max word does: interpolation is a convex combination).
 * ep_mean / ep_invstd / ep_gamma / ep_beta (nullable, eval mode; no stats / bn_part / accumulate):
 * the epilogue applies the following BatchNorm with its running statistics and the ReLU,
 * y = relu((conv + bias - mean) * invstd * gamma + beta) (srpde_bn_eval_prepare's mean / invstd),
 * so the conv output is the activation itself (models.py:22-23 in eval mode); ep_amax (nullable,
 * zeroed beforehand) receives max|y|, the next h3 consumer's operand-scale word.
 * out_max (nullable): every output tile writes max|y| of its elements to out_max[tile]
 * (ceil(P/rows) x ceil(cout/cols) slots, the h3 tile of the call) -- the scale bound that
 * srpde_bn_bwd_prepare needs when y is the gradient of a BN output.
 * in_scale / in_shift (nullable, c1 == 0 only): the input is relu(x0 * in_scale[c] + in_shift[c])
 * -- the producing BatchNorm + ReLU applied on the fly (srpde_bn_affine); padding stays zero.
 * bn_part (nullable; dgrad of a conv whose input was a BN + ReLU output, accumulate == 0): the
 * output is that activation's gradient, and the epilogue also writes the BN backward's
 * reduction, (sum dz, sum dz*xhat) per (srpde_conv_stats_rows_per_block(cout)-row block,
 * channel) into bn_part [srpde_conv_stats_blocks][cout] float2 (bn_y = the BN's input, its batch
 * mean / invstd, gamma / beta) -- for srpde_bn_relu_bwd_part */
/* weight gradient with the h3 arithmetic (same workspace as srpde_conv_wgrad; c0, c1, cout % 32 == 0);
 * amax_dy / amax0 / amax1: the max|.| words of dy, x0, x1 as for srpde_conv_fwd_h3 */
int srpde_conv_wgrad_h3(const float* dy, int lddy, const unsigned* amax_dy, const float* x0, int c0, int ldx0,
                        const unsigned* amax0, const float* x1, int c1, int ldx1, const unsigned* amax1, float* dw,
                        int cin_real, int accumulate, int n, int h, int w, int cout, int ksize, int dil,
                        void* workspace, size_t ws_bytes, hipStream_t stream);
/* h3 weight gradient from pre-split operands: dyp = the xsplit_out of the dgrad call (sign -1,
 * [2][P][cout]) or srpde_bn_bwd_apply_split's planes ([2][P][cout rounded up to 32]: cout = 16 reads
 * 32-channel planes), and xp = the xsplit_out of the forward call ([2][P][c0+c1]), with the max|.|
 * words those calls used.  No split work inside; workspace: srpde_conv_wgrad_h3p_workspace_size. */
size_t srpde_conv_wgrad_h3p_workspace_size(int n, int h, int w, int cout, int cin, int ksize);
int srpde_conv_wgrad_h3p(const void* dyp, const unsigned* amax_dy, const void* xp, int c0, const unsigned* amax0,
                         int c1, const unsigned* amax1, float* dw, int cin_real, int accumulate, int n, int h, int w,
                         int cout, int ksize, int dil, void* workspace, size_t ws_bytes, hipStream_t stream);
/* 1 when srpde_conv_wgrad_h3p runs this shape on the input-row-ring kernel for 128-channel m tiles
 * (conv_wgrad_h3g_kernel: cout 128, cin 32 .. 128 in steps of 32, w = 20, dilation 1 -- enc2.conv1 / conv2 and
 * dec2.conv2, models.py:80-81, 92); else the h3p / h3h tiles. */
int srpde_conv_wgrad_h3g_supported(int cout, int cin, int w, int dil);
/* srpde_conv_wgrad_h3p for the 40 x 40 layers (cout <= 64, c0 and c1 multiples of 32: shapes for which
 * srpde_conv_wgrad_h3x_supported returns 1) with the input read from its fp32 rows instead of a stored split,
 * so the forward need not write xsplit_out: in_scale / in_shift and x1_ca / x1_sa (nullable, in pairs) repeat
 * the forward call's input transform and amax0 / amax1 are that call's words -- the operand is bit for bit
 * the split the forward would have stored, and dw equals srpde_conv_wgrad_h3p's on it.  Workspace:
 * srpde_conv_wgrad_h3p_workspace_size. */
int srpde_conv_wgrad_h3x_supported(int c0, int c1, int cout, int w, int dil);
int srpde_conv_wgrad_h3x(const void* dyp, const unsigned* amax_dy, const float* x0, int ldx0, int c0,
                         const unsigned* amax0, const float* in_scale, const float* in_shift, const float* x1, int ldx1,
                         int c1, const unsigned* amax1, const float* x1_ca, const float* x1_sa, float* dw, int cin_real,
                         int accumulate, int n, int h, int w, int cout, int ksize, int dil, void* workspace,
                         size_t ws_bytes, hipStream_t stream);

/* ---- BatchNorm2d + ReLU -------------------------------------------------------------
 * replaces aten::native_batch_norm / native_batch_norm_backward and relu /
 * threshold_backward for every nn.BatchNorm2d (src/models.py:17,19,44,47,58,60) and the
 * F.relu / nn.ReLU after it (models.py:22-23,45,48,96-97). */
int srpde_bn_train_finalize(const float* stats, int nblk, int rows_per_blk, long long P, int C,
                            float* running_mean, float* running_var, long long* num_batches_tracked,
                            float momentum, float eps, float* mean_out, float* invstd_out, hipStream_t stream);
/* srpde_bn_train_finalize followed by srpde_bn_affine of its mean / invstd, in one launch (the same
 * outputs, bit for bit; amax_bound nullable, zeroed beforehand). */
int srpde_bn_train_finalize_affine(const float* stats, int nblk, int rows_per_blk, long long P, int C,
                                   float* running_mean, float* running_var, long long* num_batches_tracked,
                                   float momentum, float eps, float* mean_out, float* invstd_out, const float* gamma,
                                   const float* beta, float* scale, float* shift, unsigned* amax_bound,
                                   hipStream_t stream);
/* Either of the two above in two coalesced passes through a workspace of srpde_bn_finalize_workspace_size(nblk, C)
 * bytes (row slices of 16-channel groups, then one thread per channel over the slices): a 40 x 40 layer's
 * 20,480 partials per channel take a few microseconds instead of ~36.  gamma / beta / scale / shift /
 * amax_bound nullable (scale and shift together: the _affine outputs).  The fp64 sums run per slice, then over
 * the slices, so mean / invstd can differ from srpde_bn_train_finalize's in the last bit of the fp64 sums. */
size_t srpde_bn_finalize_workspace_size(int nblk, int C);
int srpde_bn_train_finalize_ws(const float* stats, int nblk, int rows_per_blk, long long P, int C, float* running_mean,
                               float* running_var, long long* num_batches_tracked, float momentum, float eps,
                               float* mean_out, float* invstd_out, const float* gamma, const float* beta, float* scale,
                               float* shift, unsigned* amax_bound, void* workspace, size_t ws_bytes,
                               hipStream_t stream);
int srpde_bn_eval_prepare(const float* running_mean, const float* running_var, int C, float eps, float* mean_out,
                          float* invstd_out, hipStream_t stream);
/* amax (nullable): *amax = max(*amax, max|out|) as float bits -- the operand-scale word of the
 * h3 convolutions; the caller zeroes it before the producing call */
int srpde_bn_relu_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                      const float* beta, float* out, int ldo, long long P, int C, int relu, unsigned* amax,
                      hipStream_t stream);
/* srpde_bn_relu_fwd of an [n][h][w][C] block output followed by srpde_maxpool2x2_fwd of it
 * (models.py:22-23 then :79-80), in one pass: out = relu(bn(y)) and pool = its 2x2 max (same
 * values and tie order as the separate calls).  h, w even. */
int srpde_bn_relu_pool_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                           const float* beta, float* out, int ldo, float* pool, int ldp, int n, int h, int w, int C,
                           int relu, unsigned* amax, hipStream_t stream);
/* srpde_bn_relu_pool_fwd (ReLU always) with one block per sample, which also forms the channel branch
 * of the AttentionGate reading the activation (models.py:106-112, 119-121; as srpde_att_channel_fwd:
 * m [n][C], hbuf [n][C/8], ca [n][C]).  C a multiple of 32, <= 256.  pool == NULL: no pooling (the
 * activation and the channel branch only).  out == NULL: the activation is not written (y already is
 * it: pass mean 0, invstd 1, gamma 1, beta 0, an exact identity on y >= 0). */
int srpde_bn_relu_pool_att_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                               const float* beta, float* out, int ldo, float* pool, int ldp, int n, int h, int w,
                               int C, unsigned* amax, const float* w1, const float* b1, const float* w2,
                               const float* b2, float* m, float* hbuf, float* ca, hipStream_t stream);
/* srpde_bn_relu_fwd (ReLU) that also forms the spatial attention of the gate whose gating input the
 * result is (models.py:124-125): sa[p] = sigmoid(sum_c wg[c] out[p][c] + bg[0]).  C 256, 512 or 1024.
 * out == NULL: the activation is not written (as srpde_bn_relu_pool_att_fwd). */
int srpde_bn_relu_gate_fwd(const float* y, int ldy, const float* mean, const float* invstd, const float* gamma,
                           const float* beta, float* out, int ldo, long long P, int C, const float* wg,
                           const float* bg, float* sa, unsigned* amax, hipStream_t stream);
/* train-mode BN folded into a per-channel affine for a consumer that applies it on the fly
 * (a = relu(y*scale + shift), srpde_conv_fwd_h3's in_scale / in_shift), plus a rigorous bound
 * on max|a| (|gamma| sqrt(P-1) + |beta|, Samuelson's inequality) into *amax_bound (nullable) */
int srpde_bn_affine(const float* mean, const float* invstd, const float* gamma, const float* beta, int C, long long P,
                    float* scale, float* shift, unsigned* amax_bound, hipStream_t stream);
size_t srpde_bn_relu_bwd_workspace_size(long long P, int C);
/* backward flags (the `relu` argument of the two calls below):
 *   SRPDE_BN_RELU  the BN output went through ReLU (mask dz by the recomputed output > 0)
 *   SRPDE_BN_EVAL  the forward normalised with the running statistics (eval mode): mean / invstd
 *                  are constants, dy = gamma*invstd*dz without the batch-statistic terms
 *                  (aten native_batch_norm_backward with training=False) */
#define SRPDE_BN_RELU 1
#define SRPDE_BN_EVAL 2
/* srpde_bn_relu_bwd with the (sum dz, sum dz*xhat) reduction already done by the producer of da
 * (srpde_conv_fwd_h3's bn_part, nblk row blocks): skips the reduction pass over y and da */
int srpde_bn_relu_bwd_part(const float* y, int ldy, const float* da, int ldda, const float* mean, const float* invstd,
                           const float* gamma, const float* beta, float* dy, int lddy, float* dgamma, float* dbeta,
                           float* dbias, long long P, int C, int relu, unsigned* amax, const void* part, int nblk,
                           void* workspace, size_t ws_bytes, hipStream_t stream);
/* The BN backward prepared for a consumer that applies it on the fly (srpde_conv_dgrad_h3_bnb):
 * dgamma, dbeta, dbias, the float vectors m1 = sum(dz)/P and m2 = sum(dz*xhat)/P, and a rigorous
 * bound on max|dy| (float bits) for the consumer's operand scale.  part (nullable): the
 * (sum dz, sum dz*xhat) partials of the dgrad that produced da, with that dgrad's per-tile
 * max|da| slots (da_max[n_da_max]); null: a reduction pass over y and da here. */
size_t srpde_bn_bwd_prepare_workspace_size(long long P, int C);
int srpde_bn_bwd_prepare(const float* y, int ldy, const float* da, int ldda, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, long long P, int C, int flags, const void* part,
                         int nblk_part, const float* da_max, int n_da_max, float* m1, float* m2, float* dgamma,
                         float* dbeta, float* dbias, unsigned* dy_amax, void* workspace, size_t ws_bytes,
                         hipStream_t stream);
/* The BN (+ReLU) backward apply with srpde_bn_bwd_prepare's m1 / m2 (the expressions of
 * srpde_bn_relu_bwd) written as the h3 operand split of dy: planes = [2][P][Cp] fp16 hi / lo of
 * dy * 2^h3_exp(*dy_amax) (dy_amax = prepare's bound), Cp = C rounded up to a multiple of 32 with
 * channels C..Cp-1 zero (out_bn2's C = 16), the input of srpde_conv_fwd_h3_presplit (c = Cp) and
 * srpde_conv_wgrad_h3p.  No fp32 dy is written. */
int srpde_bn_bwd_apply_split(const float* y, int ldy, const float* da, int ldda, const float* mean,
                             const float* invstd, const float* gamma, const float* beta, const float* m1,
                             const float* m2, long long P, int C, int flags, const unsigned* dy_amax, void* planes,
                             hipStream_t stream);
int srpde_bn_relu_bwd(const float* y, int ldy, const float* da, int ldda, const float* mean, const float* invstd,
                      const float* gamma, const float* beta, float* dy, int lddy, float* dgamma, float* dbeta,
                      float* dbias, long long P, int C, int relu, unsigned* amax, void* workspace,
                      size_t ws_bytes, hipStream_t stream);

/* ---- input staging: NCHW model input -> NHWC (channel-padded) ----------------------- */
int srpde_nchw_to_nhwc(const float* x, float* out, int n, int cin, int h, int w, int cpad, hipStream_t stream);
/* the way back for the gradient w.r.t. the model input: rows [P, ldx] -> NCHW [n, c, h, w] */
int srpde_nhwc_to_nchw(const float* x, int ldx, float* out, int n, int c, int h, int w, hipStream_t stream);
/* y[:, ch] += alpha * x for y NCHW [n, c, hw], x [n, hw] (the residual path of models.py:74,101) */
int srpde_axpy_channel(float* y, const float* x, int n, int c, int hw, int ch, float alpha, hipStream_t stream);

/* ---- nn.MaxPool2d(2)  (src/models.py:69, used :79-80) -------------------------------- */
int srpde_maxpool2x2_fwd(const float* x, int ldx, float* out, int ldo, int n, int h, int w, int c,
                         hipStream_t stream);
int srpde_maxpool2x2_bwd(const float* x, int ldx, const float* dout, int lddo, float* dx, int lddx, int n, int h,
                         int w, int c, int accumulate, hipStream_t stream);

/* ---- PDEDataset assembly (src/models.py:132-207; replaces the per-field normalisation,
 *      F.interpolate(size=fine, bilinear, align_corners=True) of the coarse field and the
 *      torch.cat of models.py:155-203) -------------------------------------------------
 * u_coarse [n][hc][wc], u_fine / theta_fine / f_fine [n][hf][wf] (contiguous fp32);
 * stats = device {u_mean, u_std, f_mean, f_std, theta_mean, theta_std} (fp32, the split's
 * statistics; theta's ignored when theta_constant != 0, theta then passes through unnormalised).
 * Writes inputs [n][3][hf][wf] = (resize((u_coarse - u_mean) / u_std), theta_n, f_n) and
 * targets [n][1][hf][wf] = (u_fine - u_mean) / u_std. */
int srpde_pde_dataset_assemble(const float* u_coarse, const float* u_fine, const float* theta_fine,
                               const float* f_fine, const float* stats, int theta_constant, int n, int hc, int wc,
                               int hf, int wf, float* inputs, float* targets, hipStream_t stream);

/* ---- bicubic, align_corners=True, single-channel fields [planes][h][w] -> [planes][ho][wo]:
 *      F.interpolate(mode='bicubic') of the cascade's interpolation baselines
 *      (src/resolution_comparison_enhanced.py:43-65 multi-level, :386-392 direct) --------- */
int srpde_resize_bicubic_ac(const float* x, float* out, int planes, int h, int w, int ho, int wo,
                            hipStream_t stream);

/* ---- bilinear, align_corners=True: nn.Upsample(2) (models.py:70, :89-93) and the
 *      F.interpolate(size=(40,40)) of PDEDataset (models.py:182-187) ------------------ */
int srpde_upsample_bilinear_fwd(const float* x, int ldx, float* out, int ldo, int n, int h, int w, int ho, int wo,
                                int c, hipStream_t stream);
int srpde_upsample_bilinear_bwd(const float* dout, int lddo, float* dx, int lddx, int n, int h, int w, int ho,
                                int wo, int c, int accumulate, hipStream_t stream);
/* srpde_upsample_bilinear_bwd of (dout + dsa (x) wg): the attention gating gradient
 * dg[q][c] += dsa[q] * wg[c] (models.py:116, srpde_att_bwd called with dg == NULL leaves dsa in
 * workspace[0, P)) folded into the upsample backward that consumes dg (models.py:89,92), so the
 * gating gradient is never written.  Needs c / 4 a power of two <= 256. */
/* srpde_upsample_bilinear_fwd that also forms the spatial attention of the gate reading the result
 * (models.py:124-125, 89/92): sa[q] = sigmoid(sum_c wg[c] out[q][c] + bg[0]).  c / 4 a power of two
 * <= 64.  With srpde_att_channel_fwd's ca, srpde_att_apply_fwd then finishes the gate. */
int srpde_upsample_bilinear_gate_fwd(const float* x, int ldx, float* out, int ldo, int n, int h, int w, int ho,
                                      int wo, int c, const float* wg, const float* bg, float* sa, hipStream_t stream);
/* The spatial attention of the gate whose gating input is up(x) (srpde_upsample_bilinear_gate_fwd's sa),
 * from the low-resolution x alone: sa[q] = sigmoid(up(x . wg)[q] + bg[0]) -- the 1x1 conv commutes with
 * the bilinear upsample, so up(x) need not exist (the decoder conv reads it through srpde_conv_fwd_h3's
 * x0_up).  Equal to the materialised form up to fp32 rounding.  workspace: n h w floats. */
size_t srpde_upsample_gate_sa_workspace_size(int n, int h, int w);
int srpde_upsample_gate_sa(const float* x, int ldx, int n, int h, int w, int ho, int wo, int c, const float* wg,
                           const float* bg, float* sa, void* workspace, size_t ws_bytes, hipStream_t stream);
/* The output head in inference, one pass (models.py:59-61, 98-101, eval mode): out[p] =
 * final(relu(bn2(out_conv2(z))))[p] + xin[n][0][q], z = [n h w][32] (row stride ldz) with its max|z|
 * word, out_conv2's h3 forward planes [2][16][288] / wexp[16] (srpde_split_weights_h3) and bias,
 * out_bn2's eval constants (srpde_bn_eval_prepare's mean / invstd, gamma, beta), final's weight [16] /
 * bias [1], xin the U-Net input (NCHW, xin_c channels).  out_conv2's values equal the h3 kernels';
 * the 16-channel dot sums in another order than srpde_head_fwd.  Replaces srpde_conv_fwd_h3 (out_conv2,
 * ep_*) + srpde_head_fwd.  Needs w <= 63. */
/* 1 if srpde_conv_head_eval takes images of width w (its halo tile needs w <= 63), else 0: wider images
 * run out_conv2 on srpde_conv_fwd_h3 and the head separately. */
int srpde_conv_head_eval_supported(int w);
int srpde_conv_head_eval(const float* z, int ldz, const unsigned* amax_z, const void* wsplit, const int* wexp,
                         const float* bias, const float* bn_mean, const float* bn_invstd, const float* bn_gamma,
                         const float* bn_beta, const float* wf, const float* bf, const float* xin, int xin_c, int n,
                         int h, int w, float* out, hipStream_t stream);
/* out[p][c] = x[p][c] * ca[n][c] * sa[p] (models.py:122, 128) */
int srpde_att_apply_fwd(const float* x, int ldx, int n, int hw, int c, const float* ca, const float* sa, float* out,
                        int ldo, hipStream_t stream);
int srpde_upsample_bilinear_bwd_gated(const float* dout, int lddo, const float* dsa, const float* wg, float* dx,
                                      int lddx, int n, int h, int w, int ho, int wo, int c, int accumulate,
                                      hipStream_t stream);
/* The same (accumulate = 0) with the backward reduction of the BatchNorm (+ ReLU, flags SRPDE_BN_RELU) whose
 * output gradient dx is -- the decoder block below the upsample (dec2.bn2 under u2, dec3.bn2 under u3,
 * models.py:88-93): y its pre-BN input, mean / invstd the batch statistics; part receives [n*h][c] float2
 * partials (sum dz, sum dz*xhat) and da_max[n*h] max|dx| per input row, the (part, da_max) pair
 * srpde_bn_bwd_prepare / srpde_bn_relu_bwd_part take, so the BN backward does not re-read dx.  Shapes:
 * srpde_upsample_bwd_bn_supported (the row-blocked kernel). */
/* The attention gate's gating gradient dg[p][c] += dsa[p] * wg[c] (srpde_att_bwd's dg pass, called with dg = NULL
 * to leave it out) fused with the backward reduction of the BN (+ ReLU) whose output gradient dg is -- the
 * bridge's last BN under att3's gating signal (models.py:46-48, 88): part [srpde_gating_bn_reduce_blocks][C]
 * float2 and da_max[blocks], the pair srpde_bn_bwd_prepare / srpde_bn_relu_bwd_part take.  C / 4 divides 256. */
int srpde_gating_bn_reduce_blocks(long long P, int C);
int srpde_gating_bn_reduce(const float* dsa, const float* wg, float* dg, int lddg, const float* y, int ldy,
                           const float* mean, const float* invstd, const float* gamma, const float* beta, long long P,
                           int C, int flags, void* part, float* da_max, hipStream_t stream);
int srpde_upsample_bwd_bn_supported(int h, int w, int ho, int wo, int c, int lddo, int lddx);
int srpde_upsample_bilinear_bwd_gated_bn(const float* dout, int lddo, const float* dsa, const float* wg, float* dx,
                                         int lddx, int n, int h, int w, int ho, int wo, int c, const float* y, int ldy,
                                         const float* mean, const float* invstd, const float* gamma,
                                         const float* beta, int flags, void* part, float* da_max,
                                         hipStream_t stream);

/* ---- AttentionGate.forward / backward (src/models.py:103-130) ----------------------- */
int srpde_att_fwd(const float* x, int ldx, const float* g, int ldg, int n, int hw, int c, int gc, const float* w1,
                  const float* b1, const float* w2, const float* b2, const float* wg, const float* bg, float* m,
                  float* hbuf, float* ca, float* sa, float* out, int ldo, hipStream_t stream);
/* srpde_att_fwd in two halves: the channel attention (mean over the pixels, the two 1x1 convs,
 * sigmoid -> ca [n][c]; depends on x alone, so it may run as soon as x exists, on another stream)
 * and the gate (spatial attention of g -> sa [n*hw], out = x * ca * sa). */
int srpde_att_channel_fwd(const float* x, int ldx, int n, int hw, int c, const float* w1, const float* b1,
                          const float* w2, const float* b2, float* m, float* hbuf, float* ca, hipStream_t stream);
int srpde_att_gate_fwd(const float* x, int ldx, const float* g, int ldg, int n, int hw, int c, int gc,
                       const float* ca, const float* wg, const float* bg, float* sa, float* out, int ldo,
                       hipStream_t stream);
size_t srpde_att_bwd_workspace_size(int n, int hw, int c, int gc);
/* dg == NULL: the gating gradient is not written; workspace[0, n*hw) floats then holds dsa (the
 * spatial gate's pre-sigmoid gradient) for srpde_upsample_bilinear_bwd_gated. */
int srpde_att_bwd(const float* dout, int lddo, const float* x, int ldx, const float* g, int ldg, int n, int hw,
                  int c, int gc, const float* w1, const float* w2, const float* wg, const float* m, const float* hbuf,
                  const float* ca, const float* sa, float* dx, int lddx, int dx_accumulate, float* dg, int lddg,
                  int dg_accumulate, float* dw1, float* db1, float* dw2, float* db2, float* dwg, float* dbg,
                  void* workspace, size_t ws_bytes, hipStream_t stream);
/* dx == NULL: the input gradient is not formed here -- workspace + n*hw floats then holds dm [n][c] (the
 * channel branch's term) for srpde_att_pool_bn_bwd. */
/* The gradient of an encoder block's output e = relu(bn(y)) that feeds both an AttentionGate (its x) and a 2x2
 * max-pool (models.py:79-80, 90/93, 119-130), and that BatchNorm's backward reduction, in one pass: de = (dout * sa)
 * * ca + dm (srpde_att_bwd's input gradient; dm from the srpde_att_bwd call with dx == NULL) plus dp [n*h/2*w/2][c]
 * routed to each 2x2 window's first maximum of a (= e; srpde_maxpool2x2_bwd's choice), written once -- bit for bit
 * srpde_att_bwd(dx) + srpde_maxpool2x2_bwd(accumulate); part [srpde_att_pool_bn_bwd_blocks()][c] float2 receives
 * (sum dz, sum dz*xhat) per block (dz = de * [bn output > 0], xhat from y, mean, invstd, gamma, beta as in
 * srpde_bn_relu_bwd) and da_max[block] max|de|: the `part` / `da_max` of srpde_bn_bwd_prepare, which then makes no
 * pass over y and de of its own.  c / 4 a power of two <= 64; h, w even. */
int srpde_att_pool_bn_bwd_blocks(int n, int h, int w, int c);
int srpde_att_pool_bn_bwd(const float* dout, int lddo, const float* ca, const float* sa, const float* dm, const float* a,
                          int lda, const float* dp, int lddp, const float* y, int ldy, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, float* de, int ldde, int n, int h,
                          int w, int c, void* part, float* da_max, hipStream_t stream);
/* The parameter-gradient half of srpde_att_bwd (dW1, db1, dW2, db2 of the channel MLP, dwg, dbg of
 * the spatial gate: fixed-order reductions over samples / pixel blocks of the per-sample rows it
 * left in `workspace`).  srpde_att_bwd with dw1 == NULL stops before it, so a caller can queue
 * these reductions on another stream (nothing downstream in the backward reads them). */
int srpde_att_bwd_params(const float* g, int ldg, int n, int hw, int c, int gc, const float* m, const float* hbuf,
                         float* dw1, float* db1, float* dw2, float* db2, float* dwg, float* dbg, void* workspace,
                         size_t ws_bytes, hipStream_t stream);
/* srpde_att_bwd_params for a gate whose gating input is the bilinear x2 upsample of d ([n*h*w][gc], the decoder
 * block's low-res output, models.py:89 / :92, hw = ho*wo the gate's resolution): the spatial conv's weight
 * gradient sum_p dsa[p] up(d)[p] is formed as sum_q d[q] (up^T dsa)[q] over the low-res rows (4x fewer bytes
 * read; the same sum regrouped, fp32 rounding apart), the bias gradient as sum_q (up^T dsa)[q]. */
int srpde_att_bwd_params_lowres(const float* d, int ldd, int n, int h, int w, int ho, int wo, int c, int gc,
                                const float* m, const float* hbuf, float* dw1, float* db1, float* dw2, float* db2,
                                float* dwg, float* dbg, void* workspace, size_t ws_bytes, hipStream_t stream);

/* ---- output head: final 1x1 conv + residual x[:,0:1] (models.py:61,74,98,101) ------- */
int srpde_head_fwd(const float* z, int ldz, int c, const float* wf, const float* bf, const float* xin, int xin_c,
                   int n, int hw, float* out, hipStream_t stream);
size_t srpde_head_bwd_workspace_size(int n, int hw, int c);
int srpde_head_bwd(const float* dout, const float* z, int ldz, int c, const float* wf, int n, int hw, float* dz,
                   int lddz, float* dwf, float* dbf, void* workspace, size_t ws_bytes, hipStream_t stream);

/* ---- nn.MSELoss (src/train_enhanced.py:70,307) --------------------------------------- */
size_t srpde_mse_workspace_size(void);
int srpde_mse_fwd(const float* y, const float* t, long long n, float* loss, void* workspace, size_t ws_bytes,
                  hipStream_t stream);
int srpde_mse_bwd(const float* y, const float* t, long long n, const float* gout, float* dy, hipStream_t stream);

/* ---- clip_grad_norm_ + AdamW on one flat buffer (src/train_enhanced.py:74-75,308) ---- */
size_t srpde_grad_norm_workspace_size(void);
int srpde_clip_coef(const float* g, long long n, float grad_scale, float max_norm, float* coef, void* workspace,
                    size_t ws_bytes, hipStream_t stream);
int srpde_adamw_step(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                     float eps, float weight_decay, int step, const float* coef, float grad_scale,
                     hipStream_t stream);

/* ---- Poisson: replaces scipy.sparse.linalg.spsolve(diag(theta) @ L, f)
 *      (src/data_generation.py:79-104, src/enhanced_data_generation.py:47-68) -------- */
int srpde_poisson_lds_max_n(void);
/* forcing f = sin(2 pi k1 X) sin(2 pi k2 Y) for B (k1, k2) pairs on linspace(0,1,n)^2
 * (PoissonSolver.generate_forcing_term, src/data_generation.py:60-77) */
int srpde_forcing_batched(const double* k12, int B, int n, double* out, hipStream_t stream);
size_t srpde_poisson_workspace_size(int B, int n);
/* The batched solve in one call (replaces spsolve(diag(theta) @ L, f), data_generation.py:79-104,
 * for B problems at once): f, theta, u are [B][n][n] fp64 device arrays, iters_out [B] int32
 * (nullable; -1 marks a problem whose cooperative launch aborted at a stuck grid barrier).
 * n <= srpde_poisson_lds_max_n(): one stream-ordered launch, no workspace.  Larger n: grid CG with
 * workspace (srpde_poisson_workspace_size bytes), run as cooperative launches (Chronopoulos-Gear CG,
 * one grid barrier per iteration, block size chosen per (B, n)) -- stream-ordered, the host never
 * waits.  Only when srpde_poisson_coop_problems(n) is 0 (n > 1024) the call drives the split entry
 * points below (textbook CG) and polls convergence every 128 iterations, synchronising `stream`. */
int srpde_poisson_cg_batched(const double* f, const double* theta, double* u, int B, int n, double rtol, int maxit,
                             int* iters_out, void* workspace, size_t ws_bytes, hipStream_t stream);
/* (Test hook: rtol < 0 solves to |rtol| but every cooperative grid-CG launch starts aborted -- iters_out = -1 for
 * its problems, u undefined -- to exercise a caller's handling of a stuck grid barrier; poisson.solve_batched
 * raises.  The LDS solver, n <= srpde_poisson_lds_max_n(), has no barrier to abort.) */
/* Problems per cooperative grid-CG launch at this n with its largest (8192-point) blocks; 0 when one
 * problem does not fit the co-resident grid or n > 1024 (a block's two halo rows, the neighbours'
 * edge rows, take at most two points per thread). */
int srpde_poisson_coop_problems(int n);
int srpde_poisson_cg_lds(const double* f, const double* theta, double* u, int B, int n, double rtol, int maxit,
                         int* iters, double* resid, hipStream_t stream);
int srpde_poisson_cg_grid_init(const double* f, const double* theta, int B, int n, void* ws, size_t ws_bytes,
                               hipStream_t stream);
int srpde_poisson_cg_grid_iterate(int B, int n, double rtol, int k_begin, int k_count, int maxit, void* ws,
                                  size_t ws_bytes, hipStream_t stream);
size_t srpde_poisson_cg_grid_done_offset(int B, int n);
int srpde_poisson_cg_grid_finish(double* u, int* iters, int B, int n, int maxit, void* ws, size_t ws_bytes,
                                 hipStream_t stream);

/* ---- Row-sharded CG for ONE n x n problem over `world` ranks (the 640^2 ground
 *      truth of solve_multi_resolution, src/resolution_comparison.py:62-73).  Rank `rank` owns the
 *      rows [row0, row0 + nloc) (rank order tiles [0, n)); f / theta / u are its [nloc][n] fp64
 *      rows.  Per iteration k the caller runs
 *        iter_a(k) -> all-gather spq (1 double per rank) into gpq[world]
 *        iter_b(k) -> all-gather send (4n + 1 doubles per rank) into gath[world][4n + 1]
 *      after init (whose send buffer is gathered first); gath / gpq may alias send / spq at world 1.
 *      Convergence (rr <= rtol^2 rr_0 or k = maxit) is decided identically on every rank; the int
 *      at byte srpde_poisson_rows_done_offset of the workspace turns nonzero then (poll it every few
 *      dozen iterations; further calls are no-ops).  No call synchronises the host. */
size_t srpde_poisson_rows_workspace_size(int n, int nloc);
size_t srpde_poisson_rows_done_offset(int n, int nloc);
int srpde_poisson_rows_init(const double* f, const double* theta, int n, int nloc, void* ws, size_t ws_bytes,
                            double* send, hipStream_t stream);
int srpde_poisson_rows_iter_a(int n, int nloc, int row0, int rank, int world, const double* gath, int k, int maxit,
                              double rtol, void* ws, size_t ws_bytes, double* spq, hipStream_t stream);
int srpde_poisson_rows_iter_b(int n, int nloc, int world, const double* gath, const double* gpq, int k, void* ws,
                              size_t ws_bytes, double* send, hipStream_t stream);
int srpde_poisson_rows_finish(double* u, int* iters, int n, int nloc, int maxit, void* ws, size_t ws_bytes,
                              hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* SRPDE_H_ */
