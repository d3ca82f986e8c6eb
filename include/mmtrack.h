/*
 * mmtrack.h — C ABI of the MI355X-native per-frame tracking engine.
 *
 * Drop-in boundary for the reference's per-frame tracker call
 * (wxltop/Multi-Modal-Trakcing-Bechmark, ViPT):
 *
 *   reference                                            this ABI
 *   ---------------------------------------------------  ---------------------------------------
 *   ViPTTrack.__init__ + build_viptrack + strict          mmt_create + mmt_set_tensor (every key)
 *     load_state_dict   (ViPT/lib/test/tracker/vipt.py:18-39,   + mmt_finalize (strict check)
 *     ViPT/lib/models/vipt/ostrack_prompt.py:94-145)
 *   ViPTTrack.initialize(image, {'init_bbox'})            mmt_initialize
 *     (vipt.py:41-62)
 *   ViPTTrack.track(image) -> {'target_bbox','best_score'} mmt_track   (one sequence)
 *     (vipt.py:64-110)                                     mmt_track_batch (N independent sequences,
 *                                                           one launch; the reference runs one
 *                                                           tracker per Pool worker,
 *                                                           RGBT_workspace/test_rgbt_mgpus.py:180-184)
 *   OSTrack.track (ViPT/lib/test/tracker/ostrack.py:75-100) same entry points, cfg.model = OSTRACK
 *   SiamFC / DiMP correlation (RGBE/models/siamfc (absent), mmt_xcorr
 *     RGBD/models/DeT/ltr/models/layers/filter.py:5-54)
 *   DiMPSteepestDescentGN.forward                          mmt_dimp_optimize
 *     (RGBD/models/DeT/ltr/models/target_classifier/optimizer.py:85-170)
 *
 * Conventions: plain pointers and sizes; frames are H x W x C uint8, row-major, channels last
 * (RGB first, then the aux modality), host or device memory; boxes are [x, y, w, h] doubles in
 * frame pixels.  Every call returns MMT_OK (0) or a negative error code; mmt_last_error() gives
 * the message (the Python mirror re-raises it with the reference's exception type and text,
 * e.g. "Too small bounding box." from processing_utils.py:34-35).  One engine owns one HIP
 * device + stream; engines are not shared between threads.
 */
#ifndef MMTRACK_H_
#define MMTRACK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mmt_engine mmt_engine;

enum {
  MMT_OK = 0,
  MMT_E_ARG = -1,      /* invalid argument (ValueError)                     */
  MMT_E_STATE = -2,    /* call out of order (e.g. track before initialize)  */
  MMT_E_HIP = -3,      /* HIP runtime failure                               */
  MMT_E_WEIGHTS = -4,  /* missing / unexpected / mis-shaped state_dict key  */
  MMT_E_BOX = -5       /* "Too small bounding box." (processing_utils.py:34-35) */
};

enum { MMT_MODEL_VIPT = 0, MMT_MODEL_OSTRACK = 1 };
enum { MMT_PROMPT_NONE = 0, MMT_PROMPT_SHAW = 1, MMT_PROMPT_DEEP = 2 };

typedef struct mmt_config {
  int model;               /* MMT_MODEL_*                                           */
  int prompt_type;         /* MMT_PROMPT_* (cfg.TRAIN.PROMPT.TYPE)                  */
  int in_chans;            /* frame channels: 6 (RGB + aux) for ViPT, 3 for OSTrack */
  int template_size;       /* cfg.TEST.TEMPLATE_SIZE (128)                          */
  int search_size;         /* cfg.TEST.SEARCH_SIZE (256)                            */
  double template_factor;  /* cfg.TEST.TEMPLATE_FACTOR (2.0)                        */
  double search_factor;    /* cfg.TEST.SEARCH_FACTOR (4.0)                          */
  int n_ce;                /* len(cfg.MODEL.BACKBONE.CE_LOC)                        */
  int ce_loc[12];
  double ce_keep_ratio[12];
  int ce_template_index;   /* CTR_POINT template token (generate_mask_cond, ce_utils.py:22-35) */
  int head_channels;       /* cfg.MODEL.HEAD.NUM_CHANNELS (256)                     */
  int max_batch;           /* sequences (slots) this engine tracks concurrently    */
  int use_graphs;          /* capture the per-frame launch sequence in a hipGraph   */
  int debug_outputs;       /* keep crops / score maps / features for parity tests   */
  int precision;           /* 1 (parity mode, what the Python tracker uses): fp32-faithful "f16x3"
                              products -- fp16 hi/lo halves of power-of-two range-scaled operands,
                              hi*hi + lo*hi + hi*lo on the fp16 MFMA: the fp32 reference's CE decisions
                              and argmax; 0: plain bf16 operands (fp32 accumulate / residual / LN /
                              softmax), ~2.3x faster, CE decisions and boxes drift from the reference */
} mmt_config;

/* lifecycle */
int mmt_create(const mmt_config* cfg, int device, mmt_engine** out);
void mmt_destroy(mmt_engine* e);
const char* mmt_last_error(const mmt_engine* e);
const char* mmt_version(void);
/* ABI revision of this header; a binding checks it once at load.  5: the strided DiMP optimiser is
 * mmt_dimp_optimize_strided (-1 = contiguous stride, 0 = broadcast; the round-3 entry point
 * mmt_dimp_optimize_dev, where 0 meant contiguous, is gone, so an old binding fails to resolve it
 * instead of silently reading sample 0 everywhere). */
#define MMT_ABI_VERSION 5
int mmt_abi_version(void);
/* pinned host memory that kernels read and write in place (mapped + coherent: a kernel sees the host's latest
 * writes and the host sees the kernel's after an event, with no copy launch) -- the DiMP pool's frame descriptors
 * and result records; NULL on failure.  mmt_host_free(NULL) is a no-op.                                     */
void* mmt_host_alloc(size_t bytes);
void mmt_host_free(void* p);

/* weights: every reference state_dict key, fp32, row-major (load_state_dict(strict=True)) */
int mmt_set_tensor(mmt_engine* e, const char* key, const float* data, const int64_t* shape, int ndim);
int mmt_finalize(mmt_engine* e);
int mmt_num_expected_keys(const mmt_engine* e);
const char* mmt_expected_key(const mmt_engine* e, int i);

/* tracking (vipt.py:41-110) */
int mmt_initialize(mmt_engine* e, int slot, const uint8_t* frame, int H, int W, int C, int64_t row_stride,
                   int is_device, const double init_xywh[4]);
int mmt_track(mmt_engine* e, int slot, const uint8_t* frame, int H, int W, int C, int64_t row_stride,
              int is_device, double out_xywh[4], float* out_score);
int mmt_track_batch(mmt_engine* e, int first_slot, int n, const uint8_t* const* frames, const int* H,
                    const int* W, int C, const int64_t* row_stride, int is_device, double* out_xywh,
                    float* out_score);
int mmt_get_state(const mmt_engine* e, int slot, double out_xywh[4]);
/* device frames (is_device = 1) are read in place on the engine's own stream: after this call every
 * initialize / track / submit with device frames first waits for the work queued so far on hip_stream
 * (the caller's producer stream, e.g. the one mmt_rgbd_assemble / mmt_rgbx_merge ran on; NULL is the
 * legacy default stream).  Without this call device frames must be complete when they are passed. */
int mmt_set_frame_stream(mmt_engine* e, void* hip_stream);
int mmt_set_state(mmt_engine* e, int slot, const double xywh[4]);

/* pipelined tracking.  The tracker state machine of ViPTTrack.track (crop geometry from the last box,
 * processing_utils.py:32-41; box back-map + clip_box, vipt.py:84-88, box_ops.py:97-106) runs on the
 * device, so a sequence's frame t+1 may be submitted before frame t's result is fetched: the host
 * round trip leaves the per-frame critical path.  mmt_track_batch == submit + fetch.
 *   submit: enqueue one frame for each of the n sequences (frames as in mmt_track_batch) -> ticket;
 *   fetch:  wait for that frame's results ('target_bbox', 'best_score' per sequence) and report its
 *           errors ("Too small bounding box." surfaces here when frames were in flight; the failing
 *           sequence keeps its state, the others advance).
 * At most MMT_PIPELINE_DEPTH submitted frames may be unfetched; initialize / set_state need none. */
#define MMT_PIPELINE_DEPTH 8
int mmt_track_batch_submit(mmt_engine* e, int first_slot, int n, const uint8_t* const* frames, const int* H,
                           const int* W, int C, const int64_t* row_stride, int is_device, int64_t* ticket);
int mmt_track_batch_fetch(mmt_engine* e, int64_t ticket, double* out_xywh, float* out_score);

/* parity / debug read-back of the last track call (debug_outputs = 1):
 *   "crop"   uint8 [S][S][C]  search patch         "maps"  f32 [5][fs*fs] ctr,size_w,size_h,off_x,off_y
 *   "feat"   f32 [Lz+Lx][768] backbone output      "removed" i32 [Lx] removed slots, CE order
 *   "result" f32 [8] cx,cy,w,h (normalised), best_score, argmax index
 *   "ce_keys" f32 [n_ce][Lx] CE score (head mean of the CTR_POINT row, attn_blocks.py:44-53) of every
 *            slot that entered each CE stage, by slot id                                        */
int mmt_debug_fetch(mmt_engine* e, const char* what, int batch_index, void* dst, size_t nbytes);
/* teacher-forced candidate elimination (parity diagnosis, debug_outputs = 1): keys [n_ce][Lx] by slot id
 * replace the engine's CE scores of `slot` in every later track call, so the reference's own scores give
 * the reference's kept sets and the remaining difference is kernel arithmetic alone.  keys = NULL turns
 * forcing off (for every slot).  Drops captured graphs.                                            */
int mmt_debug_force_ce(mmt_engine* e, int slot, const float* keys, size_t n_floats);

/* kernel timing probe: bracket every launch of one kernel class with HIP events on the engine
 * stream ("fc1", "fc2", "qkv", "proj", "attn", "conv1"); returns launches and summed ms */
int mmt_timing_enable(mmt_engine* e, const char* kernel_class);
int mmt_timing_read(mmt_engine* e, int* launches, double* total_ms, double* flops, double* bytes);

/* ---- correlation trackers (device pointers, fp32, NCHW) ---------------------------------- */
/* out[b][0][y][x] = scale * sum_c,i,j x[b][c][y+i][x+j] * z[b][c][i][j] + bias  (valid)        */
int mmt_xcorr(const float* z, const float* x, float* out, int B, int C, int hz, int wz, int hx, int wx,
              float scale, float bias, void* hip_stream);
/* the same over NHWC maps (the HIP AlexNet's layout): z [hz][wz][C] at z + b * z_batch_stride floats (0: one
 * exemplar for all B), x [B][hx][wx][C]; hz * wz * C <= 16384; 16-B aligned maps when C % 4 == 0         */
int mmt_xcorr_nhwc(const float* z, int64_t z_batch_stride, const float* x, float* out, int B, int C, int hz, int wz,
                   int hx, int wx, float scale, float bias, void* hip_stream);

/* SiamFC per-frame steps around the correlation (TrackerSiamFC.init/update, published SiamFC; the
 * reference's RGBE/models/siamfc is an empty submodule):
 *   mmt_siamfc_crop: n <= 8 square windows (top-left y0/x0, side) of a device H x W x C uint8 frame,
 *     constant border pad[3], cv2 INTER_LINEAR resize to out_sz -> out [n][3][out_sz][out_sz] float;
 *   mmt_siamfc_response: resp [n][r][r] -> INTER_CUBIC to up x up, scale penalty on scales != n/2,
 *     best scale, normalise, blend with outer(hann1d, hann1d)/hann_sum by window_influence, argmax;
 *     result (device) [4] = scale id, row, col, value; scratch: n*up*up floats (device).           */
int mmt_siamfc_crop(const uint8_t* frame, int H, int W, int C, int64_t row_stride, int n, const int* y0,
                    const int* x0, const int* size, const int pad[3], int out_sz, float* out, void* hip_stream);
/* mmt_siamfc_crop writing out [n][out_sz][out_sz][3] (NHWC, the HIP AlexNet's input)                */
int mmt_siamfc_crop_nhwc(const uint8_t* frame, int H, int W, int C, int64_t row_stride, int n, const int* y0,
                         const int* x0, const int* size, const int pad[3], int out_sz, float* out, void* hip_stream);
int mmt_siamfc_response(const float* resp, int n, int r, int up, float scale_penalty, double window_influence,
                        const double* hann1d, double hann_sum, float* scratch, float* result, void* hip_stream);

/* RGB-D frame assembly (get_rgbd_frame(..., 'rgbcolormap', depth_clip), depth_utils.py:7-58, as the
 * RGB-D VOT path calls it, vipt_class.py:79, 92): device RGB (H x W x 3 uint8) + device depth
 * (H x W uint16) -> device H x W x 6 uint8 frame (R G B | JET colormap in cv2's B G R order).
 * lut_bgr: device [256][3] colormap, or NULL for the published JET definition; workspace: device
 * buffer of mmt_rgbd_workspace_bytes() bytes.  Asynchronous on hip_stream.                       */
size_t mmt_rgbd_workspace_bytes(void);
int mmt_rgbd_assemble(const uint8_t* rgb, int64_t rgb_stride, const uint16_t* depth, int64_t depth_stride, int H,
                      int W, int depth_clip, const uint8_t* lut_bgr, uint8_t* out, int64_t out_stride,
                      void* workspace, size_t ws_bytes, void* hip_stream);

/* RGB-T / RGB-E frame assembly (get_x_frame(color, aux, dtype='rgbrgb'), depth_utils.py:71-132, as the
 * RGB-T / RGB-E workspaces call it, test_rgbt_mgpus.py:106, test_rgbe_mgpus.py:74): device RGB
 * (H x W x 3 uint8) + device aux (H x W x aux_channels uint8, 1 or 3; 1 is replicated) -> device
 * H x W x 6 uint8 frame (R G B | aux).  Asynchronous on hip_stream.                               */
int mmt_rgbx_merge(const uint8_t* rgb, int64_t rgb_stride, const uint8_t* aux, int64_t aux_stride, int aux_channels,
                   int H, int W, uint8_t* out, int64_t out_stride, void* hip_stream);

/* ---- mfDiMP / DeT-DiMP feature path (fp32, device pointers; asynchronous on hip_stream) -----------
 * The image -> classification-feature chain of DiMPnet_DeT (RGBD/models/DeT/ltr/models/tracking/
 * dimpnet.py:15-156, merge 'max') and pytracking's patch sampling; host orchestration in
 * mmtrack_amd/dimpnet.py.  Activations NHWC, conv weights [Cout][kh][kw][Cin] (BN folded).        */
#define MMT_CONV_RELU 1   /* y = max(y, 0) after bias / residual                                    */
#define MMT_CONV_MAX 2    /* y = max(y_old, y): the 'max' merge of the two backbones (dimpnet.py:103) */
#define MMT_CONV_W4 4     /* Cin == 3 and w is [Cout][kh][kw][4] (4th channel zero): the stem, one tap per load */
#define MMT_CONV_POOL 8   /* f16x3 stem (7x7 / stride 2, 4 channels, 64 outputs) with ResNet's 3x3 / stride-2 / pad-1
                             max-pool fused: y is the pooled [N][(Ho-1)/2+1][(Wo-1)/2+1][64] map (dimpnet.py backbone
                             conv1 -> bn1 -> relu -> maxpool); every group of the launch sets it or none          */
/* nn.Conv2d (+ folded BN, + residual, ReLU): y [N*Ho*Wo][Cout] = conv(x [N][H][W][Cin]); Cout % 64 == 0 */
int mmt_conv2d_f32(const float* x, int N, int H, int W, int Cin, const float* w, const float* bias, int Cout, int kh,
                   int kw, int stride, int pad, const float* resid, float* y, int flags, void* hip_stream);
/* the same with channel pitches: x pixels ldx floats apart (>= Cin), y / resid pixels ldy apart (>= Cout,
 * % 4 == 0), so one group of a grouped nn.Conv2d (groups = g) is a call at x + i*Cin, w_i, bias + i*Cout,
 * y + i*Cout (SiamFC's AlexNet, RGBE/models/siamfc); y, bias, resid 16-B aligned                     */
int mmt_conv2d_f32_ld(const float* x, int N, int H, int W, int Cin, int ldx, const float* w, const float* bias,
                      int Cout, int kh, int kw, int stride, int pad, const float* resid, float* y, int ldy, int flags,
                      void* hip_stream);
/* the same convolution on the fp16 matrix cores at fp32-faithful precision ("f16x3", csrc/dimpconv.hip):
 * w_hi / w_lo: fp16 halves of w * w_scale (w_scale a power of two with max|w| w_scale <= 2^14), layout
 * [Cout][Kp], K = kh*kw*Cin (Cin = 3: kh*kw*4, each tap padded to 4 channels), zero-padded to Kp =
 * ceil(K / 32) * 32; x_max: the input's max words (mmt_conv_max_words() floats: sharded max|x| that a
 * producing conv accumulated into its y_max) or NULL with x_scale = the static power-of-two input scale;
 * y_max: the output's max words (accumulated with agent-scope atomic max; zero them before the producer) or
 * NULL.  Cin % 32 == 0, Cin == 3, or Cin == 4 (a 3-channel image padded to 4, same weights); flags RELU /
 * MAX.                                                                                                  */
size_t mmt_conv_max_words(void);
int mmt_conv2d_f16x3(const float* x, int N, int H, int W, int Cin, const uint16_t* w_hi, const uint16_t* w_lo,
                     float w_scale, int Kp, const float* bias, int Cout, int kh, int kw, int stride, int pad,
                     const float* resid, float* y, const float* x_max, float x_scale, float* y_max, int flags,
                     void* hip_stream);
/* one convolution of a grouped f16x3 launch: the operands of mmt_conv2d_f16x3 for one of the two backbones'
 * twin layers (the same shape, their own weights, input, output and max words)                        */
typedef struct mmt_conv_group {
  const float* x;
  const uint16_t* w_hi;
  const uint16_t* w_lo;
  float w_scale;
  const float* bias;
  const float* resid;
  float* y;
  const float* x_max;
  float x_scale;
  float* y_max;
  int flags;
} mmt_conv_group;
/* the groups (1 or 2, disjoint outputs, no MAX merge when 2) in one launch; when the output tiles of the launch
 * are too few to fill the GPU, K is split in slices whose fp32 partials go to ws and are summed in slice order
 * by a second kernel that applies the epilogue (ws_bytes < mmt_conv2d_f16x3_ws_bytes(): no split)        */
size_t mmt_conv2d_f16x3_ws_bytes(int N, int H, int W, int Cin, int Cout, int kh, int kw, int stride, int pad,
                                 int groups);
int mmt_conv2d_f16x3_groups(const mmt_conv_group* groups, int n_groups, int N, int H, int W, int Cin, int Kp,
                            int Cout, int kh, int kw, int stride, int pad, void* ws, size_t ws_bytes,
                            void* hip_stream);
/* ResNet's Bottleneck tail with a downsample (resnet.py:76-95: relu(bn3(conv3(b)) + bn_d(conv_d(x)))) as ONE
 * GEMM over concatenated K: conv3 (1 x 1 over b [N][H][W][Cin]) and the downsample (1 x 1 / stride2 over the block
 * input x2 [N][H2][W2][Cin2], (H2 - 1) / stride2 + 1 == H) accumulate into the same fp32 registers, so the
 * downsample's output is never written nor read back (replaces a mmt_conv2d_f16x3_groups launch of the downsample
 * plus the conv3 launch that read it as resid).  groups[i].w_hi / w_lo: [Cout][Kp] with Kp = Cin + Cin2 -- conv3's
 * K then the downsample's, both split at the common w_scale --, bias = b3 + b_d, resid NULL; ds[i] the second
 * source (x2_max: its sharded max words, or x2_scale); the two sources are split at the smaller of their scales.
 * Cin % 32 == Cin2 % 32 == 0; workspace sized by mmt_conv2d_f16x3_ws_bytes(N, H, W, Kp, Cout, 1, 1, 1, 0, G). */
typedef struct mmt_conv_ds {
  const float* x2;
  const float* x2_max;
  float x2_scale;
} mmt_conv_ds;
int mmt_conv2d_f16x3_ds_groups(const mmt_conv_group* groups, const mmt_conv_ds* ds, int n_groups, int N, int H, int W,
                               int Cin, int H2, int W2, int Cin2, int stride2, int Kp, int Cout, void* ws,
                               size_t ws_bytes, void* hip_stream);
/* nn.MaxPool2d(k, stride, pad) over NHWC                                                           */
int mmt_maxpool2d_f32(const float* x, int N, int H, int W, int C, int k, int stride, int pad, float* y,
                      void* hip_stream);
/* NetWithBackbone.preprocess_image (net_wrappers.py:55-79): NCHW pixel values [N][C][H][W] (C = 3 or 6)
 * -> ((v / 255) - mean) / std as NHWC [N][H][W][3] per 3-channel half (out_b: the aux half)       */
int mmt_image_normalize(const float* im, int N, int C, int H, int W, const float mean[3], const float std_[3],
                        float* out_a, float* out_b, void* hip_stream);
/* the same with each pixel padded to 4 channels (a zero fourth): [N][H][W][4], what the f16x3 stem reads as one
 * 16-B load per tap (mmt_conv2d_f16x3* with Cin = 4)                                                     */
int mmt_image_normalize4(const float* im, int N, int C, int H, int W, const float mean[3], const float std_[3],
                         float* out_a, float* out_b, void* hip_stream);
/* InstanceL2Norm(size_average, eps, scale) (normalization.py:6-21) of NHWC x; y_nhwc / y_nchw may be NULL;
 * ws: device scratch of mmt_instance_l2norm_ws_bytes(N, H, W) (per-chunk sums); C % 4 == 0, C <= 1024   */
size_t mmt_instance_l2norm_ws_bytes(int N, int H, int W);
int mmt_instance_l2norm(const float* x, int N, int H, int W, int C, float scale, float eps, float* y_nhwc,
                        float* y_nchw, float* ws, void* hip_stream);
/* PrRoIPool2D(PH, PW, spatial_scale) (ltr/external/PreciseRoIPooling), roi n on image n:
 * feat NHWC, rois device [N][4] = x0, y0, x1, y1 (image coordinates) -> out [N][C][PH][PW]          */
int mmt_prroi_pool(const float* feat, int N, int H, int W, int C, const float* rois, float spatial_scale, int PH,
                   int PW, float* out, void* hip_stream);
/* sample_patch (pytracking/features/preprocessing.py:49-125) from an H x W x C uint8 device frame:
 * geom = {df, os_y, os_x, tl_y, tl_x, sz_h, sz_w} (pre-downsample factor and offset, crop top-left and
 * size in the downsampled image, replicate padding) -> bilinear resize -> float NCHW [C][out_h][out_w] */
int mmt_sample_patch(const uint8_t* frame, int H, int W, int C, int64_t row_stride, const int geom[7], int out_h,
                     int out_w, float* out, void* hip_stream);
/* one init-sample augmentation (pytracking/features/augmentation.py) of a float [C][E_h][E_w] patch,
 * cropped to out_h x out_w by crop_to_output (top / left = pad_top / pad_left, replicate)          */
#define MMT_TF_IDENTITY 0 /* Identity, Translation                                                   */
#define MMT_TF_FLIP 1     /* FlipHorizontal                                                          */
#define MMT_TF_BLUR 2     /* Blur: separable Gaussian taps fy[2 ry + 1] (vertical), fx[2 rx + 1]     */
#define MMT_TF_ROTATE 3   /* Rotate: cv2.warpAffine INTER_LINEAR / BORDER_REPLICATE, affine = the
                             inverted (dst -> src) 2 x 3 matrix                                      */
typedef struct mmt_patch_tf {
  int kind, top, left, blur_ry, blur_rx;
  float blur_fy[33], blur_fx[33];
  double affine[6];
} mmt_patch_tf;
int mmt_patch_transform(const float* img, int C, int E_h, int E_w, const mmt_patch_tf* tf, int out_h, int out_w,
                        float* out, void* hip_stream);

/* ---- DiMP / mfDiMP target classifier (device pointers, fp32) ------------------------------------
 *  feat [I][S][C][H][W] (I training images x S sequences), filter [S][C][fh][fw] (fh*fw <= 25).
 *  mmt_dimp_optimize runs num_iter steepest-descent Gauss-Newton steps in place on `weights`
 *  (DiMPSteepestDescentGN.forward, optimizer.py:85-170; relu score activation, sigmoid mask);
 *  bb: host [I][S][4] target boxes (x, y, w, h, image pixels); sample_weight: host [I][S] or NULL
 *  (= 1/I); losses: host [num_iter + 1] or NULL (when given, the call synchronises the stream). */
typedef struct mmt_dimp_params {
  float feat_stride;        /* 16                                            */
  float log_step_length;    /* optimizer.log_step_length                     */
  float filter_reg;         /* optimizer.filter_reg                          */
  float min_filter_reg;     /* 1e-3                                          */
  float alpha_eps;          /* 0                                             */
  float bin_displacement;   /* DistanceMap bin displacement                  */
  int num_dist_bins;        /* <= 128 (DiMP-50: 100)                         */
  float label_w[128];       /* label_map_predictor.weight                    */
  float mask_w[128];        /* target_mask_predictor.0.weight                */
  float spatial_w[128];     /* spatial_weight_predictor.weight               */
} mmt_dimp_params;

size_t mmt_dimp_workspace_bytes(int I, int S, int C, int H, int W, int fh, int fw, int num_iter);
int mmt_dimp_apply_filter(const float* feat, const float* w, float* scores, int I, int S, int C, int H, int W,
                          int fh, int fw, void* hip_stream);
int mmt_dimp_feat_transpose(const float* feat, const float* r, float* grad, int I, int S, int C, int H, int W,
                            int fh, int fw, void* hip_stream);
int mmt_dimp_optimize(const float* feat, int I, int S, int C, int H, int W, float* weights, int fh, int fw,
                      const float* bb, const float* sample_weight, const mmt_dimp_params* p, int num_iter,
                      void* workspace, size_t ws_bytes, float* losses, void* hip_stream);

/* ---- DiMP tracker state machine on the device (csrc/dimptrack.hip), batched over sequences ----------------
 * pytracking/tracker/dimp/dimp.py (DeT) per-frame step with the DeT_DiMP50_Max parameters, use_iou_net False:
 * the per-sequence state (position, scale, sample memory weights / boxes) lives in device memory, so a frame
 * of n sequences is: mmt_dimp_track_sample (patch geometry + sampling from the state) -> features ->
 * mmt_dimp_apply_filter -> mmt_dimp_track_update (get_sample_location, localize_advanced, update_state, memory
 * bookkeeping, the Gauss-Newton iteration choice; the frame's features into the chosen memory slot) -> the
 * host reads the n results (boxes, scores, flags, iterations) and runs mmt_dimp_optimize_strided for the
 * sequences that asked for steps.  Arrays of structs below are device memory.                          */
#define MMT_DIMP_MEMORY 50
typedef struct mmt_dimp_state {
  float pos[2], target_sz[2], base_target_sz[2], image_sz[2];   /* (y, x) as the reference's tensors       */
  float target_scale, min_scale_factor, max_scale_factor;
  int frame_num, num_init, num_stored, prev_replace;            /* prev_replace -1: None                   */
  float coords[4];                                              /* this frame's sample coords (tl, br) y,x */
  float sample_weights[MMT_DIMP_MEMORY];
  float target_boxes[MMT_DIMP_MEMORY][4];                       /* x, y, w, h in sample coordinates        */
} mmt_dimp_state;
typedef struct mmt_dimp_frame {   /* the sequence's current frame: H x W x C uint8, device                  */
  const uint8_t* data;
  int64_t stride;
  int H, W, C, pad_;
} mmt_dimp_frame;
typedef struct mmt_dimp_track_params {
  float img_sample_sz[2], feature_sz[2], kernel_size[2];
  double target_not_found_threshold, uncertain_threshold, hard_sample_threshold;   /* -inf: unset        */
  double distractor_threshold, hard_negative_threshold, target_neighborhood_scale, dispalcement_scale;
  double target_inside_ratio, low_score_opt_threshold;                             /* NaN: unset         */
  double learning_rate, hard_negative_learning_rate, init_samples_minimum_weight;   /* Python floats */
  int sample_memory_size, train_sample_interval, train_skipping;
  int net_opt_update_iter, net_opt_hn_iter, net_opt_low_iter, update_classifier;
} mmt_dimp_track_params;
typedef struct mmt_dimp_result {  /* per sequence, per frame                                                */
  float box[4];                   /* 'target_bbox' x, y, w, h                                               */
  float max_score;                /* 'confidence'                                                           */
  int flag;                       /* 0 normal, 1 not_found, 2 uncertain, 3 hard_negative                    */
  int num_iter;                   /* Gauss-Newton steps the filter takes now (0: none)                      */
  int n_samples;                  /* memory samples they run over (min(num_stored, 50))                    */
  int replace_ind;                /* memory slot written this frame (-1: none)                              */
  float tv[2], sample_pos[2], sample_scale;   /* (internal: localisation intermediates)                    */
  int aux[4];
} mmt_dimp_result;
size_t mmt_dimp_state_bytes(void);
int mmt_dimp_track_sample(mmt_dimp_state* states, const mmt_dimp_frame* frames, int n, const mmt_dimp_track_params* p,
                          int out_h, int out_w, float* patches, void* hip_stream);
/* the same patches written as the f16x3 backbones read them: each 6-channel pixel's two halves normalised
 * (((v / 255) - mean) / std, net_wrappers.py:62-72, the arithmetic of mmt_image_normalize4) into out_a / out_b
 * [n][out_h][out_w][4] (zero fourth channel) -- one launch and one patch round trip fewer than
 * mmt_dimp_track_sample + mmt_image_normalize4, the same bits.  Frames must have C == 6; `frames` may be
 * device-visible pinned host memory (read in place, no copy launch).  zero_words / n_zero (optional): floats the
 * launch clears as well (the backbones' sharded max words, cleared before their first producer).          */
int mmt_dimp_track_sample_norm4(mmt_dimp_state* states, const mmt_dimp_frame* frames, int n,
                                const mmt_dimp_track_params* p, int out_h, int out_w, const float mean[3],
                                const float std_[3], float* out_a, float* out_b, float* zero_words, int64_t n_zero,
                                void* hip_stream);
int mmt_dimp_track_update(mmt_dimp_state* states, int n, const float* scores, int sh, int sw,
                          const mmt_dimp_track_params* p, const float* feat, int64_t feat_elems, float* memory,
                          mmt_dimp_result* results, void* hip_stream);
/* the same, the records also written straight into host_results (device-visible pinned host memory) by the
 * kernel that forms them -- the host reads them after an event, without a device-to-host copy launch      */
int mmt_dimp_track_update_pinned(mmt_dimp_state* states, int n, const float* scores, int sh, int sw,
                                 const mmt_dimp_track_params* p, const float* feat, int64_t feat_elems, float* memory,
                                 mmt_dimp_result* results, mmt_dimp_result* host_results, void* hip_stream);
/* the filter updates the frame's records ask for, decided on the device: for each of the n sequences (slots
 * of states / results / filters, memory [n][MMT_DIMP_MEMORY][C][H][W]) results[s].num_iter Gauss-Newton steps
 * over its first results[s].n_samples memory samples with its state's boxes and sample weights, in one
 * launch sequence of max_iter steps (a sequence with fewer, or none, skips the rest); bitwise the filter
 * mmt_dimp_optimize_strided gives over the same samples.  Nothing comes back to the host.                   */
size_t mmt_dimp_track_optimize_ws_bytes(int n, int C, int H, int W, int fh, int fw, int max_iter);
int mmt_dimp_track_optimize(const mmt_dimp_state* states, int n, const mmt_dimp_result* results, const float* memory,
                            int C, int H, int W, float* filters, int fh, int fw, const mmt_dimp_params* p,
                            int max_iter, void* workspace, size_t ws_bytes, void* hip_stream);
/* mmt_dimp_optimize with the boxes and sample weights (or NULL) in device memory: no host staging and no
 * synchronisation (losses are not returned).  Strides in floats, -1 = the contiguous [I][S] layout (0 is a
 * real stride: one operand broadcast): sample i
 * of sequence s is feat + i * feat_img_stride + s * feat_seq_stride ([C][H][W]), its box bb_dev + i *
 * bb_img_stride + s * bb_seq_stride (4 floats), its weight sample_weight_dev[i * sw_img_stride + s * sw_seq_stride] --
 * so S sequences' memories in a pool of device states ([slot][MMT_DIMP_MEMORY] samples, mmt_dimp_state's
 * target_boxes / sample_weights) are optimised in one call, their filters weights [S][C][fh][fw].  Samples
 * with weight 0 contribute exact zeros: sequences with fewer stored samples than I give the same filter as
 * a call over their own samples.                                                                           */
int mmt_dimp_optimize_strided(const float* feat, int64_t feat_img_stride, int64_t feat_seq_stride, int I, int S,
                              int C, int H, int W, float* weights, int fh, int fw, const float* bb_dev,
                              int64_t bb_img_stride, int64_t bb_seq_stride, const float* sample_weight_dev,
                              int64_t sw_img_stride, int64_t sw_seq_stride, const mmt_dimp_params* p, int num_iter,
                              void* workspace, size_t ws_bytes, void* hip_stream);

/* ---- operator-level entry points (device pointers; used by the parity tests and by hosts that
 *      compose their own pipelines).  epi: 0 bias->bf16, 1 bias+GELU->bf16, 2 C(f32) = R + acc + bias,
 *      3 bias+ReLU->bf16, 4 bias->f32, 5 bias+ReLU->f32, 6 C(f32) = acc + bias + R[m % pos_rows].
 *      conv_hw > 0 selects the implicit 3x3 (pad 1) conv A-operand over an NHWC map.  GEMMs with few
 *      64 x 64 tiles and a long K run split-K here (fp32 partials, fixed-order reduction); the engine
 *      itself never splits K, so its results do not depend on the batch size.                     */
int mmt_op_gemm(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, void* C, int64_t ldc,
                const float* R, int64_t ldr, int M, int N, int K, int epi, int conv_hw, int conv_cin, int pos_rows,
                void* hip_stream);
int mmt_gemm_force_config(int cfg);   /* tuning: pin the dense-GEMM tile config (-1 = heuristic); 320 / 256 pin the
                                         f16x3 qkv / fc1 GEMMs to 320 x 256 / 256 x 256 tiles */
int mmt_gemm_stamps(void* dev_buf);   /* tuning: per-block s_memtime stamps [blocks][4] (start, main loop,
                                         epilogue, end) into a device buffer; NULL turns them off */
int mmt_op_attention(const void* qkv, void* out, int B, int N, int heads, int ce_query, int ce_lens_t,
                     float* ce_prob, void* hip_stream);
int mmt_op_layernorm(const float* x, const float* w, const float* b, void* out_bf16, float* out_f32, int rows,
                     void* hip_stream);
/* parity-mode ("f16x3") operators, the kernels the engine launches at precision = 1: every operand v is
 * carried as the fp16 pair hi = f16(v s), lo = f16(v s - hi) of its power-of-two range scale s
 * (uint16 storage).  GEMM: acc = sum Wh*Ah + Wl*Ah + Wh*Al, y = acc * inv + bias (inv = 1 / (s_A s_W));
 * 16-bit epilogues (0, 1, 3) write the pair of y * out_scale to C / C_lo, fp32 ones (2, 4, 5, 6) write y
 * (+ R).  Attention: qkv halves of qkv * s_qkv -> out halves of O * s_qkv (softmax scale 64^-0.5).      */
int mmt_op_gemm_f16x3(const void* A_hi, const void* A_lo, int64_t lda, const void* W_hi, const void* W_lo, int64_t ldw,
                      const float* bias, void* C, void* C_lo, int64_t ldc, const float* R, int64_t ldr, int M, int N, int K,
                      int epi, float inv, float out_scale, int conv_hw, int conv_cin, void* hip_stream);
int mmt_op_attention_f16x3(const void* qkv_hi, const void* qkv_lo, void* out_hi, void* out_lo, int B, int N, int heads,
                           int ce_query, int ce_lens_t, float* ce_prob, float s_qkv, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* MMTRACK_H_ */
