// Fused per-clip causal head of CausalAnomalyDetector (causal_anomaly_detection.py:160-502) and the step tail
// (softmax of the direct classifier, score blend cad:573-576, losses cad:673-686).
#pragma once
#include "common.h"

namespace vad {

constexpr int NMAX = 5;      // detections per frame (cad:178)
constexpr int NF_ = 6;       // num_factors
constexpr int GH = 64;       // GRU hidden
constexpr int GIN = 68;      // 4 + reid_dim

// head parameter tensors, in state_dict order
enum HeadSlot {
  H_REID0_W, H_REID0_B, H_REID2_W, H_REID2_B, H_REID4_W, H_REID4_B,
  H_GRU_WIH, H_GRU_WHH, H_GRU_BIH, H_GRU_BHH, H_ENC_W, H_ENC_B,
  H_CE0_W, H_CE0_B, H_CE2_W, H_CE2_B, H_MU_W, H_MU_B, H_LV_W, H_LV_B,
  H_SP, H_NODE_W, H_NODE_B, H_EDGE0_W, H_EDGE0_B, H_EDGE2_W, H_EDGE2_B,
  H_DYN0_W, H_DYN0_B, H_DYN2_W, H_DYN2_B, H_DYN4_W, H_DYN4_B,
  H_CS0_W, H_CS0_B, H_CS3_W, H_CS3_B, H_CS5_W, H_CS5_B,
  H_MS0_W, H_MS0_B, H_MS2_W, H_MS2_B, H_MS4_W, H_MS4_B,
  H_TS0_W, H_TS0_B, H_TS2_W, H_TS2_B, H_TS4_W, H_TS4_B,
  H_NUM
};

struct HeadArgs {
  int B, T;
  int64_t clip0;          // global index of clip 0 (RNG keying under data parallelism)
  int training;
  uint64_t h1_eps, h1_drop;
  uint32_t thr_drop;      // scorer dropout p = 0.2
  const float* pbase;     // flat parameter buffer
  int64_t off[H_NUM];     // slot offsets into pbase / grad slabs (relative to head_begin for slabs)
  int64_t head_begin;
  int lw_len;             // floats of the parameter range [off[H_ENC_W], end of the last slot) staged in LDS
  float* ws;              // per-clip workspace (small per-clip tensors)
  int64_t ws_stride;
  int* iws;               // per-clip int workspace
  int64_t iws_stride;
  float* rows;            // per-trajectory-row arrays, R = B*T*NMAX rows (see RowLayout in head.hip)
  float* grad;            // flat grad buffer (GRU / ReID weight grads are written here directly)
};

constexpr int HW_LDS = 20480;  // capacity (floats) of the sequence kernels' LDS weight image
// sets lw_len from a.off and the last slot's size; nonzero if the image does not fit or a slot is not 16-B aligned
int head_pack_weights(HeadArgs& a, const int64_t* numel);

int64_t head_ws_floats(int T);
int64_t head_iws_ints(int T);
int64_t head_rows_floats(int B, int T);

// forward: det logits [B*T][20] -> per-clip outputs
struct HeadOut {
  float* causal;   // [B]
  float* kl;       // [B]
  float* z;        // [B][5][6]
  float* adj;      // [B][6][6]
  float* boxes;    // [B][T][5][4]  valid boxes compacted per frame (fallback box when none)
  int* counts;     // [B][T]        boxes per frame (>=1)
  int* nmax;       // [B]
  int* clip_flags; // [B][2]       (any valid detection, nmax>=2)
};
int head_fwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, hipStream_t st);
// the two launches of head_fwd (row-parallel part, then the per-clip sequence part)
int head_rows_fwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, hipStream_t st);
int head_seq_fwd(const HeadArgs& a, const HeadOut& o, hipStream_t st);

// backward: upstream grads -> grad slabs [B][slab] and d(det logits) [B*T][20]
struct HeadUp {
  const float* d_causal;  // [B]
  const float* d_kl;      // [B]
  const float* d_z;       // [B][5][6] or null
  const float* d_adj;     // [B][6][6] or null
  const float* d_boxes;   // [B][T][5][4] or null: grads of the compacted per-frame detections (HeadOut::boxes)
};
int head_bwd(const HeadArgs& a, const float* det_logits, const HeadOut& o, const HeadUp& up, float* slabs,
             int64_t slab_len, float* d_det_logits, hipStream_t st);
int head_slab_reduce(const float* slabs, int B, int64_t slab_len, float* grad_head, hipStream_t st);
// GRU / ReID weight grads over all trajectory rows, written to a.grad (run after head_slab_reduce)
int head_rows_wgrad(const HeadArgs& a, hipStream_t st);

// tail: softmax(direct logits), final score, optional loss + upstream grads, flag OR-reduce
struct TailArgs {
  int B;
  const float* direct_logits;   // [B][2]
  const float* causal;          // [B]
  const float* kl;              // [B]
  const int* clip_flags;        // [B][2]
  float* probs;                 // [B][2]
  float* final_scores;          // [B]
  int* flags;                   // [2] (det_in_graph, struct_in_graph) -> also mirrored as floats
  float* flags_f;               // [2] or null
  uint64_t* det_gate;           // forward: 1 when no box is in range (no detector gradient), else 0; or null
  // loss mode
  const int64_t* labels;        // [B] or null
  float* losses;                // [5]: classification, anomaly, causal, kl, total
  // upstream grads (written when labels != null or ext grads given)
  const float* ext_d_final;     // [B]   (module API) or null
  const float* ext_d_probs;     // [B][2]
  const float* ext_d_causal;    // [B]
  const float* ext_d_kl;        // [B]
  float* d_causal;              // [B]
  float* d_kl;                  // [B]
  float* d_direct_logits;       // [B][2]
  int64_t* nbt;                 // forward: BN num_batches_tracked counters bumped (train mode) or null
  int nbt_n;
  int fwd_bwd;                  // forward with labels: also write the loss-mode upstream grads (the backward then
                                // skips its tail launch)
};
int cad_tail_fwd(const TailArgs& t, hipStream_t st);
int cad_tail_bwd(const TailArgs& t, hipStream_t st);

}  // namespace vad
