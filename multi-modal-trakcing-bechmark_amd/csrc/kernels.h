// Launch interfaces of the hand-written gfx950 kernels (host side).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace mmt {

// ---------------------------------------------------------------- GEMM (MFMA bf16 -> fp32)
// C[m][n] = epi( sum_k A[m][k] * W[n][k] + bias[n] ), A: M x K (lda), W: N x K (ldw), both bf16, K-contiguous.
enum Epi : int {
  EPI_BF16 = 0,        // bias -> bf16
  EPI_GELU_BF16 = 1,   // bias, exact GELU -> bf16
  EPI_RESID_F32 = 2,   // C(f32) = R(f32) + (acc + bias)
  EPI_RELU_BF16 = 3,   // bias, ReLU -> bf16            (head conv, BN folded)
  EPI_F32 = 4,         // bias -> f32
  EPI_RELU_F32 = 5,    // bias, ReLU -> f32
  EPI_POS_F32 = 6,     // C(f32) = (acc + bias) + R[m % pos_rows]  (OSTrack patch-embed + pos_embed)
  EPI_PARTIAL = 7,     // internal (split-K): raw fp32 partial sums into the workspace
};
enum AMode : int { A_DENSE = 0, A_CONV3 = 1 };

struct GemmGroup {
  const bf16_t* A; const bf16_t* A_lo; int64_t lda;     // A_lo: low half of the split operand (SPLIT)
  const bf16_t* W; const bf16_t* W_lo; int64_t ldw;
  const float* bias;
  void* C; void* C_lo; int64_t ldc;                     // C_lo: 16-bit outputs also emit their low half
  const float* R; int64_t ldr;
  // SPLIT ("f16x3", common.h): A / W / C halves are fp16 of range-scaled values; acc * inv = A W^T
  // (inv = 1 / (s_A s_W)) and 16-bit outputs are written as the split of value * out_scale
  float inv = 1.0f, out_scale = 1.0f;
};

struct GemmArgs {
  GemmGroup g[3];
  int groups;
  int M, N, K;
  int amode;
  int conv_hw;      // A_CONV3: feature map is conv_hw x conv_hw (NHWC rows), zero padding 1
  int conv_cin;     // A_CONV3: input channels (multiple of 64)
  int pos_rows;     // EPI_POS_F32
  int split;        // 1: fp32-faithful f16x3 products (common.h)
  int gm;           // (set by the launcher) tile rows per super-tile group of the tile order
  int ksplit;       // (set by the launcher) K splits (1: none)
  float* ws;        // split-K workspace ([groups][ksplit][M][N] fp32) or null: never split
  int64_t ws_elems; // its capacity in floats
  const bf16_t* zero;   // unused by the buffer-load kernels (kept for ABI stability of the struct)
  int defer_reduce; // EPI_RESID_F32, one group: a split-K run leaves its partial slabs for the consumer (gemm())
  int conc;         // launches of this shape running at once on the chip (the engine's stream parts; 0 / 1: alone)
};

// A residual-stream update whose split-K partial sums were left in the workspace (gemm() with defer_reduce):
// the consuming row kernel forms X[row] += sum_s ws[s][row] * inv + bias itself, with the arithmetic of the
// reduce launch it replaces (slices summed in order, then store4's EPI_RESID_F32), and writes X[row] back.
struct RowReduce {
  const float* ws;        // null: nothing pending, X is current
  int ks;                 // slabs
  int64_t slab;           // floats per slab (M * 768)
  float inv;              // f16x3 1 / (s_A s_W) (1 in bf16 mode)
  const float* bias;      // [768]
};

// returns the K splits it ran: 1, or (a.defer_reduce and few tiles) ks > 1 with the raw fp32 partial slabs left
// in a.ws ([ks][M][N], one group) for the consumer to combine (RowReduce below) instead of a reduce launch
int gemm(const GemmArgs& a, int epi, hipStream_t s);
void gemm_force_config(int cfg);   // tuning override, -1 = heuristic
int gemm_set_stamps(void* dev_buf);  // tuning: per-block cycle stamps [blocks][4] (null: off)

// ---------------------------------------------------------------- attention
struct AttnArgs {
  const bf16_t* qkv;   // [B][N][3*C]
  const bf16_t* qkv_lo;  // split mode: low halves (else null)
  bf16_t* out;         // [B][N][C]
  bf16_t* out_lo;      // split mode
  int B, N, heads;     // head dim 64, C = 64*heads
  int ce_query;        // template token whose probability row is exported (-1: none)
  int ce_lens_t;       // template length; exported keys are [ce_lens_t, N)
  float* ce_prob;      // [B][heads][N - ce_lens_t]
  // split mode (f16x3): qkv halves are fp16 of qkv * s_qkv; qk_inv = 1 / s_qkv^2, pv_inv = 1 / (2^14 s_qkv)
  // (P travels as the split of p * 2^14), out halves = split of O * out_scale
  float qk_inv = 1.0f, pv_inv = 1.0f, out_scale = 1.0f;
};
void attention(const AttnArgs& a, hipStream_t s);

// ---------------------------------------------------------------- layer norm (row of 768)
// out_bf16[r] = LN(x[src(r)]), src(r) = gather ? b*in_pitch + gather[b][t] : r ; optional copy of x[src] to xcopy[r]
// out_lo non-null: out_bf16 / out_lo are the f16x3 halves of LN * out_scale instead (common.h)
// rr.ws non-null: x[src] first receives its pending split-K update (RowReduce), written to xcopy[r] when given,
// else back to x[src] (ungathered rows only)
void layernorm(const float* x, const float* w, const float* b, bf16_t* out_bf16, bf16_t* out_lo, float out_scale,
               float* out_f32, int rows, int rows_per_seq, const int* gather, int in_rows_per_seq, float* xcopy,
               hipStream_t s, const RowReduce& rr = RowReduce{});

// ---------------------------------------------------------------- ViPT prompt blocks
struct PromptArgs {
  int layer;                 // 0: inputs are the two patch-embed outputs
  int B, Lz, Lx;             // slots per sequence = Lz + Lx
  const float* srcA;         // layer 0: tok_rgb [B][L][768]; else residual X [B][Nrows][768] (compact)
  int srcA_rows;             // rows per sequence of srcA
  const float* srcB;         // layer 0: tok_aux [B][L][768]; deep layers: unused (the previous prompt is s8)
  const int* slot2pos;       // [B][Lx] compact position (or -1) of search slots; null at layer 0
  const float* lnA_w; const float* lnA_b;   // prompt_norms[i-1] (layer 0: prompt_norms[0])
  const float* lnB_w; const float* lnB_b;   // prompt_norms[i] (layer 0 only; deep layers use fold)
  const float* w00; const float* b00;       // conv0_0 [8][768] (deep layers: LN_A's gamma / beta folded in)
  const float* w01; const float* b01;       // conv0_1 [8][768] (layer 0 only)
  const float* fold;         // deep layers: LN_B + conv0_1 folded onto the previous s8 (PromptFold)
  float smooth;              // fovea.smooth (device scalar copied to host at load)
  float* a8;                 // [B][L][8] conv0_0 branch of this layer (written)
  float* c8;                 // [B][L][8] conv0_1 branch of this layer (written)
  // deep layers: the previous prompt block's a8 / c8 and fovea smooth; its output s8 = fovea(a8) + c8 (the
  // prompt before conv1x1, onto which LN_B + conv0_1 fold) is re-formed here from them, per slot, with the
  // per-(sequence, part) softmax statistics computed in this block (fovea_stats) -- s8 is never stored
  const float* a8p; const float* c8p;
  float smooth_p;
  // deep layers: those statistics as the previous layer's LN1 formed them ([B][32], LnPromptArgs::fstat): the
  // same bits, loaded instead of re-reduced; null: computed here (fovea_stats)
  const float* fstat_p;
  RowReduce rr;              // deep layers: the previous block's fc2 split-K update of X, applied here
};
// PromptFold (float[160]) for deep layer i, from prompt_norms[i] (g, b), conv0_1 of block i (W, w0)
// and conv1x1 of block i-1 (V [768][8], v0): with V' / v0' the column-centred V / v0,
//   c8 = rstd * (Mc s + mc) + cb,  rstd = 1/sqrt(s'G s + 2 g.s + gb + eps),
//   Mc = (W diag g) V', mc = (W diag g) v0', cb = W b + w0, G = V'^T V' / 768, g = V'^T v0' / 768,
//   gb = |v0'|^2 / 768   (LN_B(P_prev) -> conv0_1, vit_ce_prompt.py:292-300, without forming P_prev)
enum { FOLD_MC = 0, FOLD_mc = 64, FOLD_cb = 72, FOLD_G = 80, FOLD_g = 144, FOLD_gb = 152, FOLD_N = 160 };
void prompt_reduce(const PromptArgs& a, hipStream_t s);

// LN1 of a block with the prompt residual fused in (writes the updated residual X and LN(X))
struct LnPromptArgs {
  int mode;                  // 1: layer 0 (X = tok_rgb + P + pos), 2: deep layer (X += P[slot])
  int rows, rows_per_seq, Lz, Lx;
  float* X;
  const float* a8; const float* c8;   // [B][Lz+Lx][8] this prompt block's branches; s8 = fovea(a8) + c8
  float smooth;
  float* fstat;              // non-null: the sequence's fovea statistics written here ([B][32], block x = 0)
  const float* w1; const float* b1;         // conv1x1 channel-major [8][768] -> the prompt P = w1^T s8 + b1
  const float* tok_rgb;      // mode 1
  const float* pos;          // mode 1: [Lz+Lx][768]
  const int* gidx;           // mode 2: [B][rows_per_seq - Lz] slot of each compact search token
  const float* w; const float* b;
  bf16_t* out; bf16_t* out_lo;   // out_lo non-null: f16x3 halves of LN * out_scale
  float out_scale;
};
// the fovea statistics of the row's sequence, s8 of its slot, the prompt residual (conv1x1 of s8, formed per
// row from an LDS copy of conv1x1) and LN1, for the compact rows
void prompt_expand_ln(const LnPromptArgs& a, hipStream_t s);
// a deep layer's prompt_reduce (pa) and prompt_expand_ln (la, mode 2) as one launch whose blocks meet at a
// per-sequence barrier (bar: [B][32] ints, zero at allocation, left zero); false: not taken (the caller launches the two)

// ---------------------------------------------------------------- candidate elimination
struct CEArgs {
  int B, Lz, Ls, keep, heads, Lx;
  const float* prob;      // [B][heads][Ls]
  const int* gidx_in;     // [B][Ls] slot id of compact search token
  int* gidx_out;          // [B][keep]
  int* gather;            // [B][Lz + keep] source compact row of each new row
  int* slot2pos;          // [B][Lx] updated
  int* removed;           // [B][Lx] removed slot ids, appended at removed_off
  int removed_off;
  // parity diagnostics (null in production):
  const float* forced;    // [B][Lx] keys by slot id replacing the head-mean scores (teacher-forced CE:
                          // the reference's own scores give the reference's kept set)
  float* keys_out;        // [B][Lx] the head-mean score of every surviving slot, by slot id
  int keys_pitch;         // floats between sequences of forced / keys_out
};
void ce_select(const CEArgs& a, hipStream_t s);
// ce_select + the LN2 that gathers the survivors (layernorm with a.gather), one launch for few sequences; false:
// not taken (the caller launches the two)
bool ce_layernorm(const CEArgs& a, const float* x, const float* w, const float* b, bf16_t* out_bf16, bf16_t* out_lo,
                  float out_scale, int in_rows_per_seq, float* xcopy, hipStream_t s, const RowReduce& rr);

// final norm + token recovery (zeros at pruned slots) -> head input NHWC bf16 [B][Lx][768]
// feat_lo non-null: feat / feat_lo are the f16x3 halves of the normed rows * feat_scale
void final_norm_recover(const float* X, int rows_per_seq, const int* slot2pos, const float* w, const float* b,
                        int B, int Lz, int Lx, bf16_t* feat, bf16_t* feat_lo, float feat_scale, float* feat_f32_dbg,
                        hipStream_t s, const RowReduce& rr = RowReduce{});

// ---------------------------------------------------------------- crop + normalise + patchify
struct TrackOut {                  // one per sequence of a launch (read back by the host)
  double box[4];                   // 'target_bbox' after this frame (unchanged state on error)
  float score;                     // 'best_score'
  int err;                         // 0, or the geometry error of this frame
  int pad_[2];
};
struct CropParam {                 // one per sequence (device memory, rewritten every frame)
  const uint8_t* frame;            // H x W x C uint8, row stride in bytes
  int64_t stride;
  int H, W, C;
  int x1, y1, crop_sz;             // processing_utils.py:32-41
  int pad_;
};
struct SeqState;
struct RingArgs {
  const CropParam* params;   // device-visible pinned [kring][pitch]
  TrackOut* outs;            // device-visible pinned [kring][pitch] (decode writes the launch's results)
  int* ctr;                  // launches so far mod kring (device; the ring entry of the next launch)
  int* cur;                  // ring entry of the launch in flight (device)
  int kring, pitch;
};
struct GeomArgs {                  // crop_kernel<FUSED_GEOM>: the geometry kernel's operands (state null: not fused)
  SeqState* state;
  double factor;
  RingArgs ring;
  int use_ring;
  int* gidx; int* slot2pos;
  int Lz, Lx;
};
struct CropArgs {
  const CropParam* params;         // [B]
  int B, out_sz, C;                // C = 6 (RGB+aux) or 3
  bf16_t* A_rgb; bf16_t* A_aux;    // [B][rows_per_seq][768]
  bf16_t* A_rgb_lo; bf16_t* A_aux_lo;  // split mode (else null): A / A_lo are the f16x3 halves of the
                                       // normalised pixel * kPixScale
  int rows_per_seq, row0;          // patch rows land at row0 + patch index
  uint8_t* dbg_patch;              // optional [B][out][out][C]
  GeomArgs geom;                   // state non-null: the crop geometry formed in this launch (no geometry_kernel)
};
void crop_patchify(const CropArgs& a, hipStream_t s);
constexpr float kPixScale = 4096.0f;   // |(p/255 - mean) / std| <= 2.64: 2^12 keeps the f16x3 halves below 2^14

// ---------------------------------------------------------------- head tail + decode
// ---------------------------------------------------------------- device-resident tracker state
// The per-sequence state machine of ViPTTrack.track (vipt.py:64-88) lives on the device, so a
// sequence's next frame can be enqueued before this frame's box is read back: the crop geometry is
// derived from the last box on the device (geometry_kernel) and the box back-map + clip_box run in
// the decode kernel.  Doubles and rounding exactly as the reference's python / tensor mix.
struct SeqState {                  // one per slot
  double box[4];                   // self.state [x, y, w, h]
  double rf;                       // resize_factor of the frame being tracked
  int err;                         // MMT_E_BOX / MMT_E_ARG of this frame's geometry, else 0
  int pad_;
};
// processing_utils.py:32-41 for the search crop of sequences [0, n): params[i] <- x1, y1, crop_sz of
// state[i].box (factor, out_sz), state[i].rf <- out_sz / crop_sz, state[i].err <- geometry error.
// Ring hand-off (ring non-null): the frame fields of params[i] are first read from the host's pinned
// ring entry ring->params[(ctr % kring) * pitch + i] (no copy launch), then *cur <- that entry and
// ctr advances -- one per launch, in the same order as the host's tickets.
// (gidx / slot2pos non-null: also the launch's token index arrays, [n][Lx] each, as before any elimination)
void crop_geometry(CropParam* params, SeqState* state, int n, double factor, int out_sz, const RingArgs* ring,
                   int* gidx, int* slot2pos, int Lz, int Lx, hipStream_t s);

struct DecodeArgs {
  int B, fs;                       // feature map fs x fs
  const float* h4;                 // [3][B][fs*fs][32]  (ctr, offset, size) conv4 outputs (ReLU'd)
  const float* w5;                 // [5][32]: ctr, off_x, off_y, size_w, size_h
  const float* b5;                 // [5]
  const float* hann;               // [fs*fs]
  float* res;                      // [B][8]: cx, cy, w, h, score, idx
  float* maps;                     // optional [B][5][fs*fs] (ctr, size w/h, offset x/y)
  // tracker-state update (vipt.py:84-88, box_ops.py:97-106); null state: result rows only
  SeqState* state;                 // [B]
  const CropParam* params;         // [B] frame H / W of this frame
  TrackOut* out;                   // [B]
  int search_size;
  TrackOut* ring_outs;             // ring hand-off (or null): out rows also go to ring_outs[*ring_cur * pitch + row0 + b]
  const int* ring_cur;
  int ring_pitch, row0;
  int* ring_ctr;                   // non-null (the crop formed the geometry): advance the ring counter, mod ring_kring
  int ring_kring;
};
void decode(const DecodeArgs& a, hipStream_t s);

// ---------------------------------------------------------------- SiamFC / DiMP correlation
// out[b][y][x] = scale * sum_{c,i,j} X[b][c][y+i][x+j] * Z[b][c][i][j] + bias   (valid, fp32)
void xcorr(const float* Z, const float* X, float* out, int B, int C, int hz, int wz, int hx, int wx, float scale,
           float bias, hipStream_t s);
// the same over NHWC feature maps (the layout of the HIP AlexNet backbone): z [hz][wz][C] per batch entry at
// z + b * z_bstride (0: one exemplar for every entry), x [B][hx][wx][C]
void xcorr_nhwc(const float* Z, int64_t z_bstride, const float* X, float* out, int B, int C, int hz, int wz, int hx,
                int wx, float scale, float bias, hipStream_t s);

// ---- SiamFC (siamfc.hip)
struct SiamCropArgs {
  const uint8_t* frame;            // H x W x C uint8 (C >= 3; the first 3 channels are used)
  int64_t stride;
  int H, W, C;
  int n, out_sz;                   // crops, output side
  int y0[8], x0[8], size[8];       // window corner (may lie outside the frame) and side, per crop
  int pad[3];                      // border colour (cv2 Scalar -> uint8)
  float* out;                      // [n][3][out_sz][out_sz], or [n][out_sz][out_sz][3] when nhwc
  int nhwc;
};
void siamfc_crop(const SiamCropArgs& a, hipStream_t s);

struct SiamRespArgs {
  const float* resp;               // [n][r][r]
  int n, r, up;                    // scales, response side, upsampled side
  float penalty, one_minus_wi;
  double wi, hann_sum;             // cosine window = outer(hann1d, hann1d) / hann_sum (np.hanning, float64)
  const double* hann1d;            // [up] (device)
  float* scratch;                  // [n][up][up]
  float* result;                   // [4] scale id, row, col, windowed response max
};
void siamfc_response(const SiamRespArgs& a, hipStream_t s);

}  // namespace mmt
