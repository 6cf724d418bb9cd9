/*
 * libvadhip — C ABI of the MI355X (gfx950) hot path of
 * pvvkishore/Causal-Learning-Based-Video-Anomaly-Detection_Paper_Code_Raw.
 *
 * The reference exposes no FFI: its boundary is the Python nn.Module surface
 * (SURVEY.md §8b).  Every entry point below replaces one piece of that surface;
 * the Python package binds them with ctypes.
 *
 * Conventions
 *   - all pointers are DEVICE pointers unless stated; fp32 unless stated;
 *   - `stream` is a hipStream_t passed as void*; every call only enqueues work;
 *   - return 0 on success, non-zero on error; vad_last_error() has the text
 *     (the Python layer raises RuntimeError, mirroring cad:702-709);
 *   - the caller (PyTorch) owns every buffer, including the workspace.
 */
#ifndef VAD_H_
#define VAD_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VAD_ABI_VERSION 1

int vad_abi_version(void);
const char* vad_last_error(void);

/* ------------------------------------------------------------------------------------------
 * RNG (bit-exact twin of oracle/rng.py).  Replaces the torch CPU generator draws of
 * nn.Dropout and torch.randn_like in the reference (cad:170,173,330,438,528,531).
 * ------------------------------------------------------------------------------------------ */
/* uint32 u24 draws for rows row0.. and cols 0..ncols-1 (testing the contract) */
int vad_rng_u24(uint64_t seed, uint32_t stream_id, uint64_t step, int64_t row0, int64_t nrows, int64_t ncols,
                uint32_t* out, void* stream);
/* synthetic clips: x = (u8 - 0.5) / 0.5, u8 = hash >> 56 (UCSDped2Dataset + Normalize(0.5,0.5), cad:92-96) */
int vad_synth_frames(uint64_t seed, uint64_t step, int64_t frame0, int64_t nframes, int64_t npix, int mode,
                     float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * causal_anomaly_detection.py — CausalAnomalyDetector (cad:508-586) + train_model step (cad:609-690)
 * ------------------------------------------------------------------------------------------ */
typedef struct vad_cad_plan vad_cad_plan;

/* flat parameter layout: slot i = i-th entry of model.named_parameters() (state_dict order) */
int vad_cad_num_slots(void);
const char* vad_cad_slot_name(int i);
int64_t vad_cad_slot_numel(int i);
int64_t vad_cad_slot_offset(int i);
/* 0 frozen (cad:596-598), 1 always has grad, 2 detector (grad iff any in-range box), 3 structure learner
 * (grad iff some clip has >=2 trajectories), 4 never has grad (structure_params) */
int vad_cad_slot_group(int i);
int64_t vad_cad_param_floats(void);   /* flat params size; the grad buffer has 256 extra floats (flags) */
int vad_cad_num_bufs(void);           /* BatchNorm running_mean / running_var tensors, state_dict order */
const char* vad_cad_buf_name(int i);
int64_t vad_cad_buf_numel(int i);
int64_t vad_cad_buf_offset(int i);
int64_t vad_cad_buf_floats(void);
int vad_cad_num_bn(void);             /* num_batches_tracked counters (int64 array) */

int vad_cad_create(int B, int T, int H, int W, vad_cad_plan** out);
void vad_cad_destroy(vad_cad_plan* plan);
int64_t vad_cad_workspace_bytes(const vad_cad_plan* plan);
/* bind caller-owned buffers. exp_avg/exp_avg_sq/steps may be NULL when no optimizer step is used. */
int vad_cad_bind(vad_cad_plan* plan, void* workspace, float* params, float* grads, float* bufs, int64_t* nbt,
                 float* exp_avg, float* exp_avg_sq, int32_t* steps);

/* CausalAnomalyDetector.forward.  training=1: batch-stat BN + running-stat update + dropout.
 * labels (int64 [B], may be NULL) additionally computes the train_model loss terms.
 * outputs: final [B], probs [B,2], causal [B], kl [B], z [B,5,6], adj [B,6,6], nmax int32 [B],
 *          boxes [B,T,5,4], counts int32 [B,T], losses [5] (cls, anomaly, causal, kl, total), flags int32 [2] */
int vad_cad_forward(vad_cad_plan* plan, const float* x, int training, uint64_t seed, uint64_t step, int64_t clip0,
                    const int64_t* labels, float* final_scores, float* probs, float* causal, float* kl, float* z,
                    float* adj, int32_t* nmax, float* boxes, int32_t* counts, float* losses, int32_t* flags,
                    void* stream);
/* backward of the last forward.  use_loss=1: upstream grads of the train_model loss (needs labels in forward);
 * otherwise the given upstream grads (any may be NULL = zero).  Writes the flat grad buffer (all slots). */
int vad_cad_backward(vad_cad_plan* plan, int use_loss, const float* d_final, const float* d_probs,
                     const float* d_causal, const float* d_kl, const float* d_z, const float* d_adj, void* stream);
/* vad_cad_backward in two calls (same arguments; stage 0 then stage 1, both on the same stream): stage 0 runs the
 * loss tail, the causal head, the direct classifier and the detector and zeroes the grad buffer first, so every
 * grad outside the backbone slots is final when it returns; stage 1 runs the backbone (cad:141-158).  Replaces
 * the single `total_loss.backward()` (cad:688) when a data-parallel caller overlaps the head-grad all-reduce with
 * the backbone backward (DDP's bucketed reduce during backward). */
int vad_cad_backward_stage(vad_cad_plan* plan, int stage, int use_loss, const float* d_final, const float* d_probs,
                           const float* d_causal, const float* d_kl, const float* d_z, const float* d_adj,
                           void* stream);
/* stage 2 of vad_cad_backward_stage is stage 0 for a caller that orders its own consumer of the non-backbone grads
 * itself: it returns as soon as the caller's stream has its part queued, the causal head / detector backward keeps
 * running on the plan's side stream, and stage 1 (the backbone) then waits only for the detector's input gradient;
 * vad_cad_wait_side(plan, s) makes stream s wait for everything queued so far on that side stream (a data-parallel
 * caller's all-reduce stream, before it sums those grads).  Stage 1 after stage 2 re-joins the side stream. */
int vad_cad_wait_side(vad_cad_plan* plan, void* stream);
/* vad_cad_wait_layer_grads(plan, l, s): stream s waits until every grad of backbone layer l (0..7: the conv weight and
 * bias and the BatchNorm gamma / beta of causal_anomaly_detection.py:128-139's l-th conv; layer 0 also the stem's) of
 * the backbone backward queued last is final -- the per-layer buckets of a data-parallel gradient all-reduce, issued
 * while the layers below are still in their backward (DDP's reduce-during-backward, cad:688-690). */
int vad_cad_wait_layer_grads(vad_cad_plan* plan, int layer, void* stream);
/* vad_cad_input_ready(plan, s) arms the NEXT vad_cad_forward of this plan (one-shot): its input clips are complete
 * once the work queued on stream s at this call is.  With the frozen fused stem (and per-rank BatchNorm statistics)
 * that forward then runs conv1 + bn1 + the max pool on a plan stream ordered after that point only -- not after
 * what the caller's stream still has queued, e.g. the previous step's last weight gradient and optimizer step --
 * and layer1.0 waits for it.  Without the call a forward orders its stem after the caller's stream, as before.
 * (No reference counterpart: the reference's forward is synchronous, cad:669-690.) */
int vad_cad_input_ready(vad_cad_plan* plan, void* stream);
/* vad_cad_backward_stage with one more upstream grad: d_boxes [B,T,5,4] (may be NULL), the grad of a loss on the
 * forward's compacted per-frame detections (boxes output of vad_cad_forward; the reference's detections are slices
 * of the rescaled detector output and carry autograd, cad:201-222).  The constant fallback box takes no grad. */
int vad_cad_backward_ext(vad_cad_plan* plan, int stage, int use_loss, const float* d_final, const float* d_probs,
                         const float* d_causal, const float* d_kl, const float* d_z, const float* d_adj,
                         const float* d_boxes, void* stream);
/* clip_grad_norm_(max_norm) + AdamW over the flat buffers (torch.optim.AdamW semantics, per-slot steps,
 * slots without a grad this step are skipped).  grad_scale multiplies grads first (1/world for DP).
 * total_norm (device float [1], may be NULL) receives the pre-clip norm. */
int vad_cad_optimizer_step(vad_cad_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                           float max_norm, float grad_scale, float* total_norm, void* stream);
/* SyncBatchNorm mode (BASELINE config 3 parity with the reference's single-process global batch: its BatchNorm2d
 * layers normalise over all B*T frames, cad:116,131,136).  In training mode each of the nine BN layers folds its
 * partial sums into a per-plan double buffer `sums` ([2*C]: forward sum(x) | sum(x^2); backward sum(dZ) |
 * sum(dZ*xhat)) and calls fn(user, bn_layer 0..8, phase 0 fwd / 1 bwd, n_doubles, stream); fn must replace the
 * buffer by its sum over the process group (an all-reduce ordered on `stream`) and return 0.  Statistics then use
 * world * local count.  The buffer's address: vad_cad_debug_buffer(plan, "bn_sync").  fn NULL = per-rank BN
 * (DDP default). */
typedef int (*vad_bn_sync_fn)(void* user, int bn_layer, int phase, int64_t n, void* stream);
int vad_cad_set_bn_sync(vad_cad_plan* plan, vad_bn_sync_fn fn, void* user, int world);

/* ------------------------------------------------------------------------------------------
 * Single building blocks (kernel unit tests; same kernels as the fused step)
 * ------------------------------------------------------------------------------------------ */
/* Y[M,N] = act(X[M,K] W[N,K]^T + b)  (nn.Linear + optional ReLU) */
int vad_dense_forward(const float* X, int M, int K, const float* W, const float* b, int N, float* Y, int relu,
                      float* scratch, int64_t scratch_floats, void* stream);
/* nn.Conv2d(Ci, Co, 3, stride, padding=1) on NHWC activations; W in torch layout [Co][Ci][3][3].
 * scratch: wf/wd 9*Ci*Co floats each, partials >= ceil(M/64)*2*Co floats (M = NF*OH*OW). */
int vad_conv3x3_forward(const float* x_nhwc, int NF, int Ci, int IH, int IW, const float* w, const float* bias,
                        int Co, int stride, float* y_nhwc, float* wf_scratch, float* wd_scratch, float* partials,
                        void* stream);
/* input gradient of the same conv (transposed conv; stride-2 split into four parity classes) */
int vad_conv3x3_dgrad(const float* dy_nhwc, int NF, int Ci, int IH, int IW, const float* w, int Co, int stride,
                      float* dx_nhwc, float* wf_scratch, float* wd_scratch, void* stream);
/* kernel tuning knobs (sweeps): "conv_fwd_tile", "conv_dgrad_tile", "conv_wgrad_tile" (tile id 0..9, -1 = built-in
 * choice), "conv_wgrad_blocks", "conv_wgrad_min_ktiles".  Process-global. */
int vad_set_tuning(const char* key, int value);
/* weight gradient of the same conv: dW[Co][Ci][3][3] = sum over pixels dY x patches(x); split-K slabs in partial */
int vad_conv3x3_wgrad(const float* x_nhwc, const float* dy_nhwc, int NF, int Ci, int IH, int IW, int Co, int stride,
                      float* dW, float* partial, int64_t partial_floats, void* stream);
/* the backbone's BatchNorm backward apply pass (cad:116,131,136 -- the per-element half of BatchNorm2d + ReLU
 * backward): dY = k (dZ - mean dZ - xhat mean(dZ xhat)), dZ = dA [s y + t > 0]; rows M = NF*H*W, channels C;
 * stats = the layer's [7 C] state [mean | invstd | scale | shift | k | mean dZ | mean dZ xhat]; bf16 != 0: dA, y, dY
 * are bf16 (config 4), else fp32 */
int vad_bn_bwd_apply(const void* dA, const void* y, const float* stats, int M, int C, void* dY, int bf16,
                     void* stream);

/* ------------------------------------------------------------------------------------------
 * minicausal_vad_complete3.py — SimpleVideoAnomalyDetector (mc:25-102) + StableTrainer step (mc:249-330)
 * replaces: model(data) (mc:272), criterion(outputs, targets) (mc:284), loss.backward() (mc:292), the grad
 * NaN check / norm / conditional clip (mc:294-306) and optimizer.step() (mc:308, Adam lr 1e-3 wd 1e-5, mc:229-234)
 * ------------------------------------------------------------------------------------------ */
typedef struct vad_mc_plan vad_mc_plan;

/* x: (B, C, T, H, W) fp32 NCDHW (torch layout) */
int vad_mc_create(int B, int C, int T, int H, int W, vad_mc_plan** out);
void vad_mc_destroy(vad_mc_plan* plan);
/* slot i = i-th entry of model.named_parameters(); buffers = BatchNorm3d running stats (state_dict order) */
int vad_mc_num_slots(const vad_mc_plan* plan);
const char* vad_mc_slot_name(const vad_mc_plan* plan, int i);
int64_t vad_mc_slot_numel(const vad_mc_plan* plan, int i);
int64_t vad_mc_slot_offset(const vad_mc_plan* plan, int i);
int64_t vad_mc_param_floats(const vad_mc_plan* plan);
int vad_mc_num_bufs(const vad_mc_plan* plan);
const char* vad_mc_buf_name(const vad_mc_plan* plan, int i);
int64_t vad_mc_buf_numel(const vad_mc_plan* plan, int i);
int64_t vad_mc_buf_offset(const vad_mc_plan* plan, int i);
int64_t vad_mc_buf_floats(const vad_mc_plan* plan);
int64_t vad_mc_workspace_bytes(const vad_mc_plan* plan);
/* nbt: int64[3] num_batches_tracked; steps: int32[num_slots] Adam step counters */
int vad_mc_bind(vad_mc_plan* plan, void* workspace, float* params, float* grads, float* bufs, int64_t* nbt,
                float* exp_avg, float* exp_avg_sq, int32_t* steps);
/* scores: (B,) sigmoid outputs.  labels (B,) fp32 nullable -> BCE.  losses (nullable, float[4]): bce, grad norm,
 * clipped (0/1), status (0 skipped: non-finite outputs/loss; 1 counted, no step: non-finite grads; 2 stepped) —
 * the last three are filled by vad_mc_optimizer_step.  Dropout keys: (seed, step, clip0 + b). */
int vad_mc_forward(vad_mc_plan* plan, const float* x, int training, uint64_t seed, uint64_t step, int64_t clip0,
                   const float* labels, float* scores, float* losses, int32_t* flags, void* stream);
/* d_scores (B,) nullable: NULL = backward of the forward's BCE (requires labels) */
int vad_mc_backward(vad_mc_plan* plan, const float* d_scores, void* stream);
/* grad norm (float64 sum of per-param norm^2); clip_grad_norm_(max_norm) only when norm > clip_above; Adam */
int vad_mc_optimizer_step(vad_mc_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                          float clip_above, float max_norm, void* stream);

/* ------------------------------------------------------------------------------------------
 * avenue_training_script2.py — a2 CausalAnomalyDetector (a2:15-101), compute_improved_loss (a2:135-205) and the
 * ImprovedMiniCausalVAD step (a2:218-245).  replaces: self.model(videos) (a2:224), compute_improved_loss (a2:227),
 * loss.backward() (a2:235), clip_grad_norm_(0.5) (a2:236), AdamW(lr 5e-4, wd 1e-3).step() (a2:115-119, 238)
 * ------------------------------------------------------------------------------------------ */
typedef struct vad_a2_plan vad_a2_plan;

int vad_a2_num_slots(void);            /* 20 = model.named_parameters() order (188,849 parameters) */
const char* vad_a2_slot_name(int i);
int64_t vad_a2_slot_numel(int i);
int64_t vad_a2_slot_offset(int i);
int64_t vad_a2_param_floats(void);
/* x: (B, 3, T, H, W) fp32 NCDHW, 2 <= B <= 256 */
int vad_a2_create(int B, int T, int H, int W, vad_a2_plan** out);
void vad_a2_destroy(vad_a2_plan* plan);
int64_t vad_a2_workspace_bytes(const vad_a2_plan* plan);
int vad_a2_bind(vad_a2_plan* plan, void* workspace, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                int32_t* steps);
/* outputs (nullable): scores (B,), adj (B,16,16), features (B,16).  with_loss: compute_improved_loss with
 * pseudo-labels keyed (seed, step, clip0 + b); losses float[10]: total, anomaly, acyclicity, sparsity,
 * consistency, structure, edge_count, sparsity_ratio, grad norm (optimizer), status (0 NaN skip, 2 stepped) */
int vad_a2_forward(vad_a2_plan* plan, const float* x, int training, uint64_t seed, uint64_t step, int64_t clip0,
                   int with_loss, float* scores, float* adj, float* features, float* losses, void* stream);
/* "borrow_input" 1: the next forwards read x in place and the backward reads it again (the caller keeps it unchanged
 * until then, as the fused train step does); 0 (default): the forward copies x for conv3d_1's weight gradient */
int vad_a2_set_option(vad_a2_plan* plan, const char* key, int64_t value);
/* compute_improved_loss alone, on the last forward's scores / adjacency (pseudo-labels keyed by seed/step/clip0);
 * vad_a2_loss_grads copies d total / d scores (B,) and d total / d adj (B,16,16) of that loss */
int vad_a2_loss(vad_a2_plan* plan, uint64_t seed, uint64_t step, int64_t clip0, float* losses, void* stream);
int vad_a2_loss_grads(vad_a2_plan* plan, float* d_scores, float* d_adj, void* stream);
/* all upstream grads NULL: backward of the forward's loss; else the given (nullable) output grads */
int vad_a2_backward(vad_a2_plan* plan, const float* d_scores, const float* d_adj, const float* d_features,
                    void* stream);
int vad_a2_optimizer_step(vad_a2_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                          float max_norm, void* stream);

/* ------------------------------------------------------------------------------------------
 * avenue_training_script_bbox.py — CausalAnomalyDetector forward (bbox:51-101), eval mode, as run by
 * AnomalyVisualizer.predict_anomaly_for_clip (bbox:339-368).  replaces: self.model(video_tensor) (bbox:357)
 * ------------------------------------------------------------------------------------------ */
typedef struct vad_bbox_plan vad_bbox_plan;

int vad_bbox_num_slots(void);          /* 12 = model.named_parameters() order */
const char* vad_bbox_slot_name(int i);
int64_t vad_bbox_slot_numel(int i);
int64_t vad_bbox_slot_offset(int i);
int64_t vad_bbox_param_floats(void);
/* x: (B, 3, T, H, W) fp32 NCDHW, one clip length per plan (mixed-T batches: one plan per T) */
int vad_bbox_create(int B, int T, int H, int W, vad_bbox_plan** out);
void vad_bbox_destroy(vad_bbox_plan* plan);
int64_t vad_bbox_workspace_bytes(const vad_bbox_plan* plan);
int vad_bbox_bind(vad_bbox_plan* plan, void* workspace, const float* params);
/* scores (B,), adj (B,16,16), features (B,1024, nullable) */
int vad_bbox_forward(vad_bbox_plan* plan, const float* x, float* scores, float* adj, float* features, void* stream);

/* ------------------------------------------------------------------------------------------
 * causal_anomaly_detection1.py — memory-bank VideoAutoEncoder (cad1:124-321) and the train_model iteration
 * (cad1:372-431).  replaces: model(videos) (cad1:392), reconstruction_loss (cad1:400), model.update_memory
 * (cad1:407), total_loss.backward() (cad1:411), the NaN-grad check + clip_grad_norm_(0.1) + Adam.step()
 * (cad1:413-425), and the eval forwards of the validation / calculate_anomaly_scores loops (cad1:460, 542-552)
 * ------------------------------------------------------------------------------------------ */
typedef struct vad_ae_plan vad_ae_plan;

int vad_ae_num_slots(void);            /* 38 = model.named_parameters() order */
const char* vad_ae_slot_name(int i);
int64_t vad_ae_slot_numel(int i);
int64_t vad_ae_slot_offset(int i);
int64_t vad_ae_param_floats(void);
int vad_ae_num_bufs(void);             /* 14 BatchNorm running_mean / running_var tensors, state_dict order */
const char* vad_ae_buf_name(int i);
int64_t vad_ae_buf_numel(int i);
int64_t vad_ae_buf_offset(int i);
int64_t vad_ae_buf_floats(void);
/* clips (B, T, 1, 64, 64) fp32 (the encoder's Linear(128*4*4) fixes 64x64 frames), 1 <= B <= 500 */
int vad_ae_create(int B, int T, vad_ae_plan** out);
void vad_ae_destroy(vad_ae_plan* plan);
int64_t vad_ae_workspace_bytes(const vad_ae_plan* plan);
/* nbt: int64[7] num_batches_tracked (encoder.1/4/7/10, decoder.4/7/10); memory: float[500*64] normal_memory;
 * memory_ptr: int64[1]; exp_avg / exp_avg_sq / steps (int32[num_slots]) may be NULL until an optimizer step */
int vad_ae_bind(vad_ae_plan* plan, void* workspace, float* params, float* grads, float* bufs, int64_t* nbt,
                float* memory, int64_t* memory_ptr, float* exp_avg, float* exp_avg_sq, int32_t* steps);
/* stages: 3 = forward() (encode_sequence + decode_sequence + compute_anomaly_score), 1 = encode_sequence only,
 * 2 = decode_sequence of seq_in (B, 64) over T frames.  loss_mode (stages 3): 0 none; 1 the reconstruction MSE
 * against x and per-clip errors (eval loops); 2 the train_model iteration: MSE and its gradient, a non-finite input
 * skips the batch without touching BN running stats / counters / the ring (cad1:385-387), a valid batch's sequence
 * features enter the ring after the scores (cad1:407).  Outputs (nullable): recon (B,T,1,64,64), seq (B,64),
 * frame_feats (B,T,64), scores (B,), recon_err (B,) (loss_mode > 0).  losses float[4]: mse, grad norm, clipped,
 * status (0 skipped, 1 non-finite grads, 2 stepped; the middle two and the final status from the optimizer) */
int vad_ae_forward(vad_ae_plan* plan, const float* x, const float* seq_in, int stages, int training, int loss_mode,
                   float* recon, float* seq, float* frame_feats, float* scores, float* recon_err, float* losses,
                   void* stream);
/* backward of the last full forward: use_loss = 1 -> of its train_model MSE, else the given output grads
 * (nullable = zero).  Writes every slot of the flat grad buffer. */
int vad_ae_backward(vad_ae_plan* plan, int use_loss, const float* d_recon, const float* d_seq,
                    const float* d_frame_feats, void* stream);
/* non-finite-grad skip, clip_grad_norm_(max_norm) and Adam with coupled L2 weight decay (cad1:350-351, 413-425);
 * grad_scale multiplies the grads first (1/world after a data-parallel sum) */
int vad_ae_optimizer_step(vad_ae_plan* plan, float lr, float beta1, float beta2, float eps, float weight_decay,
                          float max_norm, float grad_scale, void* stream);
/* the memory ring of any VideoAutoEncoder: update_memory (cad1:201-219; n <= 500 features (n, 64)) and
 * compute_anomaly_score (cad1:262-301; n sequence features -> scores (n,)) */
/* test access to the last forward's pre-activations (the gradient tests pin their LeakyReLU decisions): "ey" idx l:
 * encoder conv l's raw output [T*B frames, t-major][H][W][Co]; "est" idx l: its per-frame-index BN state [T][8][Co]
 * (mean | invstd | scale | shift | ...); "dy" idx j < 3: decoder ConvTranspose2d j's raw output [B][H][W][Co]; "dst"
 * idx j: its BN state [8][Co]; "u": the decoder Linear's output [B][2048].  Device pointers (vad_debug_d2h). */
int vad_ae_debug_buffer(vad_ae_plan* plan, const char* name, int idx, void** ptr, int64_t* nfloats);
int vad_ae_update_memory(float* memory, int64_t* memory_ptr, const float* features, int n, void* stream);
int vad_ae_memory_score(const float* memory, const int64_t* memory_ptr, const float* seq, int n, float* scores,
                        void* stream);

/* Host data path.
 * vad_u8_to_clip: n u8 pixels -> fp32; mode 0: (u8 - 0.5) / 0.5 (UCSDped2Dataset + Normalize, cad:85-104,
 *   1177-1179), mode 1: u8 / 255 (ToTensor, mc:120 / bbox:411).  src (in HBM, or pinned host memory at the address
 *   vad_host_device_ptr gives) and dst 16-byte aligned.
 * vad_host_device_ptr: the device address of pinned host memory (the ClipStager's direct mode reads batches there).
 * vad_resize_u8 (host): bilinear u8 resize, half-pixel centres, clamped borders, 11-bit fixed-point weights (the
 *   cv2.resize INTER_LINEAR scheme of cad:88-89). */
int vad_u8_to_clip(const uint8_t* src, int64_t n, int mode, float* dst, void* stream);
int vad_host_device_ptr(const void* host, void** dev);
int vad_resize_u8(const uint8_t* src, int sh, int sw, uint8_t* dst, int dh, int dw);

/* Plan options.  "conv_bf16" (0/1): the 3x3 convs of the backbone run on bf16 operands with fp32 accumulation
 * (BASELINE config 4's bf16 compute; BN, pooling, heads, losses and the optimizer stay fp32).  Default 0: fp32
 * numerics (split-bf16 products).  "stem_grad" (0/1): backbone.conv1 / bn1 train (the module without
 * apply_memory_efficient_training, cad:592-598); set before the forward.  "wgrad_stream" (0/1, default 1): the
 * backbone's weight gradients run on a plan-owned stream beside the input gradients (results identical). */
int vad_cad_set_option(vad_cad_plan* plan, const char* key, int64_t value);
/* Kernel family of backbone 3x3 conv `layer` (0..7) for kind 0 forward / 1 input gradient / 2 weight gradient:
 * 6 = split-bf16 (fp32 numerics, six bf16 MFMA products per K step), 1 = bf16 operands, 0 = f32 MFMA; -1 on error.
 * (bench.py prices each launch against the peak of the instruction mix it runs.) */
int vad_cad_conv_path(vad_cad_plan* plan, int layer, int kind);

/* ------------------------------------------------------------------------------------------
 * Debug introspection (tests only): internal plan buffers, partial backward, device->host copy
 * names: y1, pool, y[0..7], stats[0..8], feats, pooled, dA, dY, d_pooled, d_feat_det, det_logits
 * ------------------------------------------------------------------------------------------ */
int vad_cad_debug_buffer(vad_cad_plan* plan, const char* name, int idx, void** ptr, int64_t* nfloats);
int vad_cad_set_debug(vad_cad_plan* plan, const char* key, int64_t value);  /* "stop_layer" */
int vad_debug_d2h(void* host, const void* dev, int64_t bytes);
/* HIP-event timing of labelled launches (conv_fwd/L<l>, conv_wgrad/L<l>, conv_dgrad/L<l>, bn_bwd_*, conv1,
 * det_fwd, head_fwd, optimizer, ...).  enable: 0 pauses (records kept), 1 clears the records and starts, 2 starts
 * appending.  only_prefix restricts the labels recorded; with a non-empty prefix the labelled conv kernels are
 * dispatched with their own start/stop events (hipExtLaunchKernel) instead of event records around the launch. */
int vad_cad_profile(vad_cad_plan* plan, int enable, const char* only_prefix);
int vad_cad_profile_read(vad_cad_plan* plan, char* labels, double* total_ms, int* counts, int cap);
/* per-record label / start / end (ms after the first record), record order (bench.py: the post-backbone chain) */
int vad_cad_profile_marks(vad_cad_plan* plan, char* labels, double* t0_ms, double* t1_ms, int cap);

#ifdef __cplusplus
}
#endif
#endif /* VAD_H_ */
