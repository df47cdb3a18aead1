/* libllp_hip.so — C ABI of the MI355X (gfx950) LLP distillation hot path.
 *
 * Every entry point takes caller-owned DEVICE pointers (row-major, contiguous
 * unless a leading dimension says otherwise), plain sizes, and the HIP stream
 * to launch on as `void* stream` (a hipStream_t; NULL = legacy stream).  No
 * entry point allocates, frees or synchronises, so every call can be captured
 * into a hipGraph.  Return 0 on success, else an LLP_E_* / hipError_t code;
 * llp_last_error() gives a thread-local message.
 *
 * The reference (snap-research/linkless-link-prediction) is pure Python; it
 * has no C ABI of its own.  Each entry point names the reference operation it
 * replaces (file:line, paths relative to the reference root).
 */
#ifndef LLP_HIP_H_
#define LLP_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LLP_OK 0
/* A ticket block (the one-launch loss, gradient norm, compaction and dense-negative scans):
 * LLP_TICKET_WORDS uint32, zero before the first call, returned to zero by every call. */
#define LLP_TICKET_WORDS 2080
#define LLP_E_ARG 10001
#define LLP_E_WORKSPACE 10002

enum llp_dtype { LLP_F32 = 0, LLP_BF16 = 1,
                 /* aux of llp_gemm_nt only: a ReLU bit mask, bit c%8 of byte c/8 of row r at
                  * aux + r*ld_aux (bytes) -- written by an act=RELU GEMM (bit = bf16 output > 0),
                  * read by act=RELU_BWD in place of the bf16 activations (16x less traffic) */
                 LLP_MASK = 2 };

enum llp_act {
  LLP_ACT_NONE = 0,      /* y = alpha*acc + bias                          */
  LLP_ACT_RELU = 1,      /* y = max(alpha*acc + bias, 0)                  */
  LLP_ACT_RELU_BWD = 2   /* y = (alpha*acc + bias) * (aux > 0): the ReLU
                            backward fused into a dgrad GEMM's epilogue    */
};

/* A GEMM operand: logical row r (0 <= r < rows) is
 *   ptr[(idx ? idx[r] : r) * ld + k]                       (plain / gathered)
 *   ptr[(idx ? idx[r] : r) * ld + k] * ptr2[(idx2 ? idx2[r] : r) * ld2 + k]
 *                                                          (Hadamard, ptr2 != NULL)
 * Element type is the GEMM's dtype.  This is how the build avoids
 * materialising x[this_target] (src/main.py:95-96) and x_i*x_j
 * (src/models.py:140). */
typedef struct llp_operand {
  const void* ptr;
  const int32_t* idx;
  const void* ptr2;
  const int32_t* idx2;
  int64_t ld;
  int64_t ld2;
  /* Optional device-resident row count (int32, may be NULL).  When set, the
   * GEMM runs on min(M, *rows_dev) rows (llp_gemm_nt: of A and C; llp_gemm_tn:
   * the contraction rows of A and B) while its grid stays sized by the host M,
   * so a data-dependent row count (the unique-node student, *n_unique of
   * llp_dedup_rows) needs no host read and the launch is hipGraph-capturable. */
  const int32_t* rows_dev;
} llp_operand;

int llp_version(void);
const char* llp_last_error(void);
/* Name of the NT GEMM kernel the last llp_gemm_nt / llp_gemm_nt_head call on this thread
 * launched (thread-local, "" before the first): the bench labels its roofline kernel with it. */
const char* llp_last_gemm_kernel(void);
/* 1 if the HIP runtime sees a device (never required to load the library). */
int llp_device_count(void);

/* ---------------------------------------------------------------- GEMM (MFMA)
 * C[m,n] = epi(alpha * sum_k A[m,k] * B[n,k]),  m<M, n<N, k<K.
 * Replaces nn.Linear forward (src/models.py:48,143,146) with B = weight [N,K],
 * and the data-gradient dX = dY . W with B = W^T.  dtype LLP_F32 runs the exact
 * f32 MFMA (v_mfma_f32_16x16x4_f32); LLP_BF16 runs v_mfma_f32_16x16x32_bf16
 * with f32 accumulation.  c_dtype / aux_dtype select the output / aux element
 * type (aux_dtype LLP_MASK: aux is a ReLU bit mask, see enum llp_dtype; bf16
 * 256-tile path only).  bias (f32[N]) may be NULL. */
/* Optional inverted dropout after the activation (F.dropout / nn.Dropout after
 * ReLU, src/models.py:52-53,144-145): element (m, n) is kept iff its keep
 * draw (8 bits when p*256 is an integer, else 16; one Philox block per 16 or 8
 * elements of a row, layout in csrc/llp_common.h drop_keep, oracle
 * dropout_keep) in Philox stream 64*(*step_ctr) + stream_offset is >= the
 * threshold p*256 (8-bit) or ceil(p*65536) (16-bit); kept values are scaled by
 * 1/(1-p).
 * The backward needs no mask: LLP_ACT_RELU_BWD against the stored dropped
 * activation with alpha = 1/(1-p) is exact. */
typedef struct llp_dropout {
  float p;
  uint64_t seed;
  const int64_t* step_ctr;
  int64_t stream_offset;
} llp_dropout;

int llp_gemm_nt(int dtype, int64_t M, int64_t N, int64_t K,
                const llp_operand* A, const llp_operand* B,
                void* C, int64_t ldc, int c_dtype,
                const float* bias, int act, const void* aux, int64_t ld_aux, int aux_dtype,
                float alpha, const llp_dropout* dropout, void* stream);

/* bf16 GEMM with the LinkPredictor's last Linear(N, 1) fused into the epilogue
 * (src/models.py:143-146): y = act(alpha * A.B^T + bias) (+dropout) is stored to
 * C (C may be NULL when only the head is needed) and each 256-column tile t
 * writes head_part[t][m] = sum_{n in tile} y[m, n] * head_w[n] (f32, exact
 * activations before bf16 rounding).  llp_head_finish sums the
 * llp_gemm_nt_head_parts(N) partials in a fixed order, adds the bias and
 * applies torch.sigmoid (src/models.py:150). */
int64_t llp_gemm_nt_head_parts(int64_t N);
int llp_gemm_nt_head(int64_t M, int64_t N, int64_t K, const llp_operand* A, const llp_operand* B,
                     void* C, int64_t ldc, const float* bias, int act, float alpha,
                     const llp_dropout* dropout, const float* head_w, float* head_part, void* stream);
/* The same for f32 operands (the fp32 path, the reference's arithmetic): C = relu(A.B^T + bias) f32
 * (stored: the head backward reads it) and head_part[N / 256][M] = the Linear(N,1) head's partial
 * dots over each 256-column tile, summed in a fixed order (src/models.py:143-146).  Plain 16-B
 * aligned f32 operands, K % 64 == 0, N % 256 == 0; finish with llp_head_finish (+ bias). */
int llp_gemm_nt_head_f32(int64_t M, int64_t N, int64_t K, const llp_operand* A, const llp_operand* B, float* C,
                         int64_t ldc, const float* bias, const float* head_w, float* head_part, void* stream);
int llp_head_finish(int64_t parts, int64_t M, const float* part, const float* b, float* logit,
                    float* prob, void* stream);

/* Split-K bf16 GEMM for few output tiles over a long K: the first Linear of the
 * full-batch student (src/models.py:48 on x [N_old, 8,415] at the coauthor-physics
 * production shape, src/main.py:173), where C = act(A.B^T + bias) has fewer
 * 256x256 tiles than the CUs.  Workgroup (tile, s) sums K-tiles
 * [nkt*s/S, nkt*(s+1)/S) into an f32 slab of `workspace`
 * (llp_gemm_nt_splitk_ws_bytes), then one pass sums the S slabs in order, adds the
 * bias, rounds to bf16 and applies act (NONE or RELU, with an optional ReLU bit
 * mask as llp_gemm_nt writes it).  Deterministic; equal to llp_gemm_nt up to where
 * the K-range partial sums are added.  llp_gemm_nt_splitk_plan returns S (1: use
 * llp_gemm_nt).  bf16 only; plain, 16-B aligned operands; N % 256 == 0. */
int llp_gemm_nt_splitk_plan(int64_t M, int64_t N, int64_t K);
int64_t llp_gemm_nt_splitk_ws_bytes(int64_t M, int64_t N, int splits);
int llp_gemm_nt_splitk(int64_t M, int64_t N, int64_t K, const llp_operand* A, const llp_operand* B,
                       void* C, int64_t ldc, const float* bias, int act, void* mask_out, int64_t ld_mask,
                       int splits, void* workspace, int64_t workspace_bytes, void* stream);


/* Weight gradient: C[p,q] (+)= sum_m A[m,p] * B[m,q]  (A = dY [M,P], B = X [M,Q]).
 * Split over m into slabs in `workspace` (llp_gemm_tn_workspace_bytes), then
 * reduced in a fixed order: deterministic.  C is f32 with leading dim ldc.
 * colsum_a (f32[P], may be NULL) (+)= sum_m A[m,p]: the bias gradient, fused
 * into the same pass over dY.  Replaces autograd's weight/bias gradient of
 * nn.Linear (src/main.py:132). */
int64_t llp_gemm_tn_workspace_bytes(int dtype, int64_t M, int64_t P, int64_t Q);
int llp_gemm_tn(int dtype, int64_t M, int64_t P, int64_t Q,
                const llp_operand* A, const llp_operand* B,
                float* C, int64_t ldc, int accumulate, float* colsum_a,
                void* workspace, int64_t workspace_bytes, void* stream);
/* llp_gemm_tn with the output's columns split between two matrices: columns [0, q_split) to C
 * (row stride ldc), columns [q_split, Q) to C2 (C2 column 0 = column q_split, row stride ldc2).
 * One weight-gradient GEMM over a K-concatenated operand [agg(x) | x] written straight into a
 * SAGEConv's lin_l and lin_r gradients (src/sageconv_updated.py:65-81; PyG SAGEConv via
 * src/models.py:110-119).  0 < q_split < Q; same workspace as llp_gemm_tn. */
int llp_gemm_tn_split(int dtype, int64_t M, int64_t P, int64_t Q,
                      const llp_operand* A, const llp_operand* B,
                      float* C, int64_t ldc, int64_t q_split, float* C2, int64_t ldc2,
                      int accumulate, float* colsum_a,
                      void* workspace, int64_t workspace_bytes, void* stream);

/* Sparse-input first Linear (src/models.py:48 on bag-of-words x, e.g. coauthor-physics' 8,415
 * binary keywords at ~0.5 % density; csrc/spmm.hip).  x is held as CSR (rowptr[N+1], colidx,
 * val; val NULL = all ones) and, per student slice, as CSC (colptr[F+1], rowidx ascending within
 * a column, local to the slice).  Wt is the bf16 transposed weight [F, H] (row stride ldw).
 *   llp_spmm_rows: Y[r, :] = act(sum_{k in CSR row row0 + r} val[k] * Wt[colidx[k], :] + bias)
 *                  for r < rows, bf16 out (RNE), act NONE or RELU, optional ReLU bit mask as
 *                  llp_gemm_nt writes it (the next layer's ReLU-backward GEMM reads it).
 *   llp_spmm_tn:   dW[o, f] (+)= sum_{k in CSC column f} val[k] * dY[rowidx[k], o]: the
 *                  weight gradient of the same Linear (f32, row stride ldw >= F); the bias
 *                  gradient is llp_colsum of dY.
 * f32 sums in a fixed order (forward: 4 interleaved streams of the row's nonzeros, summed
 * (s0+s1)+(s2+s3); backward: 8 interleaved streams, butterfly-summed, over a column's nonzeros
 * or, for a heavy column, over each of 4 contiguous quarters, then (q0+q1)+(q2+q3)): deterministic, equal to llp_gemm_nt /
 * llp_gemm_tn on the dense x up to the order of the f32 sums.  H <= 4096, H % 8 == 0, 16-B
 * aligned rows of Wt, Y and dY.  Column slices go to XCDs by workgroup index (csrc/spmm.hip). */
int llp_spmm_rows(int64_t rows, int64_t row0, int64_t H, const int32_t* rowptr, const int32_t* colidx,
                  const float* val, const void* Wt, int64_t ldw, const float* bias, int act, void* Y,
                  int64_t ldy, void* mask_out, int64_t ld_mask, void* stream);
int llp_spmm_tn(int64_t F, int64_t H, const int32_t* colptr, const int32_t* rowidx, const float* val,
                const int32_t* perm, int64_t n_heavy, const void* dY, int64_t ldy, float* dW, int64_t ldw,
                int accumulate, void* stream);
/* The same two operations for Wt / Y / dY of either dtype (LLP_BF16 as above, or LLP_F32: f32
 * rows in and out, the same order of f32 sums; the fp32 engine's sparse first layer, whose
 * arithmetic is the reference's own; src/models.py:48).  The ReLU bit mask is bf16-only. */
int llp_spmm_rows_dt(int dtype, int64_t rows, int64_t row0, int64_t H, const int32_t* rowptr,
                     const int32_t* colidx, const float* val, const void* Wt, int64_t ldw, const float* bias,
                     int act, void* Y, int64_t ldy, void* mask_out, int64_t ld_mask, void* stream);
int llp_spmm_tn_dt(int dtype, int64_t F, int64_t H, const int32_t* colptr, const int32_t* rowidx,
                   const float* val, const int32_t* perm, int64_t n_heavy, const void* dY, int64_t ldy,
                   float* dW, int64_t ldw, int accumulate, void* stream);
/* llp_spmm_tn's schedule: perm = the features by nonzero count, most first (ties by index); the
 * first n_heavy (>= llp_spmm_heavy_nnz() nonzeros) take a workgroup each, split in quarters
 * summed (q0+q1)+(q2+q3); the rest one wave each. */
int llp_spmm_heavy_nnz(void);

/* Column sums: out[n] (+)= sum_m Y[m,n] (bias gradient).  Deterministic. */
int64_t llp_colsum_workspace_bytes(int64_t M, int64_t N);
int llp_colsum(int dtype, int64_t M, int64_t N, const void* Y, int64_t ldy, float* out, int accumulate,
               void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- link-predictor head
 * logit[r] = dot(Z[r,:], w) + b; prob[r] = sigmoid(logit[r]) (either may be NULL).
 * The last Linear(H,1) + torch.sigmoid of LinkPredictor (src/models.py:146,150),
 * or the whole 'inner' predictor (src/models.py:147-148) with w = NULL (sum). */
int llp_head_fwd(int dtype, int64_t R, int64_t H, const void* Z, int64_t ldz,
                 const void* Z2, int64_t ldz2, const int32_t* iz, const int32_t* iz2,
                 const float* w, const float* b, float* logit, float* prob, void* stream);

/* Backward of the head: dZ[r,n] = alpha * dlogit[r] * w[n] * (Z[r,n] > 0)  (ReLU (+dropout: alpha = 1/(1-p)) of the
 * layer below fused; relu_mask=0 disables the mask), dw[n] (+)= sum_r dlogit[r]*Z[r,n],
 * db (+)= sum_r dlogit[r].  dw/db reductions are deterministic slabs. */
int64_t llp_head_bwd_workspace_bytes(int64_t R, int64_t H);
int llp_head_bwd(int dtype, int64_t R, int64_t H, const float* dlogit, const void* Z, int64_t ldz,
                 const float* w, int relu_mask, float alpha, void* dZ, int64_t lddz, float* dw, float* db,
                 int accumulate, void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- fused LLP loss
 * One wavefront per anchor b (src/main.py:98-130):
 *   s = sigmoid(s_logit[b,:]) (Q4), t = t_prob[b,:];
 *   LLP_D = sum_b KL(softmax(t/T) || softmax(s/T)) * T^2 / B          (main.py:27-31)
 *   LLP_R = mean over b and pairs i<j of max(0, -y_ij (s_i - s_j) + margin),
 *           y = +1 if t_i > t_j + margin, -1 if t_i < t_j - margin, else 0 (main.py:109-122)
 *   BCE   = mean_r BCE(sigmoid(out_logit[r]), r < n_pos)                (main.py:125-127)
 *   loss  = w_label*BCE + w_d*LLP_D + w_r*LLP_R                         (main.py:129-130)
 * dlogit_ctx[b,c] / dlogit_lab[r] receive d(loss_scale*loss)/d(logit).
 * Normalisers are explicit (B_total, n_lab_total) so a rank holding a shard
 * computes its share of the global mean (multi-GPU).  terms_out (f32[4]) =
 * {loss, bce, llp_d, llp_r} partial sums of this call, written (accumulate=0)
 * or added (accumulate=1) deterministically. */
int64_t llp_llp_loss_workspace_bytes(int64_t B, int64_t n_lab);
int llp_llp_loss(int64_t B, int64_t C, const float* s_logit, const float* t_prob,
                 int64_t n_lab, int64_t n_pos, const float* out_logit,
                 double B_total, double n_lab_total, float margin, float T,
                 float w_label, float w_d, float w_r, float loss_scale,
                 float* dlogit_ctx, float* dlogit_lab, float* terms_out, int accumulate,
                 const int32_t* neg_count, int64_t neg_offset, double pos_total,
                 void* workspace, int64_t workspace_bytes, void* stream);
/* llp_llp_loss with a term range (round 4; llp_llp_loss keeps its round-3 signature and
 * reports every anchor, [0, B)).
 * [term_b0, term_b1): the anchors whose KL / rank terms enter terms_out (every anchor's
 * gradient is written): with the owner decomposition every rank evaluates the loss of
 * all B anchors on the all-reduced logits and reports the terms of its own slice
 * (llp_pair_owner_assign); [0, B) otherwise.
 * neg_count (may be NULL): the PyG-dense negatives' device count of the whole batch
 * (llp_neg_sample_dense), so the full-batch step needs no host read of it.  The label
 * rows are then n_pos positives and n_lab - n_pos negative SLOTS holding columns
 * [neg_offset, ...) of the whole batch's negatives; a slot at or past *neg_count is inert
 * (zero gradient, no loss), and the BCE mean runs over pos_total + *neg_count labels
 * (n_lab_total unused). */
int llp_llp_loss_range(int64_t B, int64_t C, const float* s_logit, const float* t_prob,
                       int64_t n_lab, int64_t n_pos, const float* out_logit,
                       double B_total, double n_lab_total, float margin, float T,
                       float w_label, float w_d, float w_r, float loss_scale,
                       float* dlogit_ctx, float* dlogit_lab, float* terms_out, int accumulate,
                       const int32_t* neg_count, int64_t neg_offset, double pos_total,
                       int64_t term_b0, int64_t term_b1,
                       void* workspace, int64_t workspace_bytes, void* stream);

/* llp_llp_loss in ONE launch, with the Linear(H, 1) heads finished inside it
 * (llp_head_finish's fixed-order sum: bit-identical logits).  s_head (may be NULL): the
 * student predictor's gemm_nt_head partials over its B*C + n_lab rows (contexts, then labels):
 * logit of row m = *bias + sum_t part[t * ld + m], written to s_logit[m] (m < B*C) and
 * out_logit[m - B*C]; NULL: the logits are read from those buffers.  t_head (may be NULL):
 * the teacher predictor's partials over the B*C context rows; t_prob[m] = sigmoid(logit),
 * written.  ticket (may be NULL: a separate finalize launch follows): a ticket block
 * (LLP_TICKET_WORDS); the workgroup that arrives last sums the partials of terms_out.  Replaces src/main.py:103-130 (head, sigmoid, losses). */
typedef struct llp_head_parts {
  const float* part;   /* [parts][ld] f32 */
  const float* bias;   /* [1] or NULL */
  int64_t parts, ld;
} llp_head_parts;
int llp_llp_loss_heads(int64_t B, int64_t C, float* s_logit, float* t_prob,
                       int64_t n_lab, int64_t n_pos, float* out_logit,
                       double B_total, double n_lab_total, float margin, float T,
                       float w_label, float w_d, float w_r, float loss_scale,
                       float* dlogit_ctx, float* dlogit_lab, float* terms_out, int accumulate,
                       const int32_t* neg_count, int64_t neg_offset, double pos_total,
                       int64_t term_b0, int64_t term_b1,
                       const llp_head_parts* s_head, const llp_head_parts* t_head, uint32_t* ticket,
                       void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- multi-rank owner decomposition
 * The N-rank form of train_minibatch's pairs (src/main.py:86-130; the reference is single-GPU):
 * each predictor pair goes to exactly one rank, the owner of its key node (owner = owner_tab[node]
 * in [0, world), or node / ceil(N / world) when owner_tab is NULL), balanced so that rank r gets cap_r = (r+1)n/world - rn/world pairs of each
 * category (an owner keeps its first cap_r pairs in item order; the owners' overflow, in
 * (owner, position) order, fills the ranks' free positions in rank order).  Category c's
 * ends: item i's node e[(i / kc) * kld + koff + (i % kc) * kstep] (a context pair (b, k): a = the
 * anchor samples[b, 0] (kc = C, kld = C + 1, koff = kstep = 0), b = samples[b, 1 + k] (koff =
 * kstep = 1), key_b = 1; a label pair: a = src, b = dst (kc = kld = 1, koff = kstep = 0), key_b = 0).
 * sel [sum n]: rank r's items of category c at sel[sum_{c'<c} n_c' + r n_c / world + j];
 * gpos [sum n] (may be NULL): item -> its slot (minus the category base); target [2 R2]
 * (may be NULL): this rank's pairs, categories in order, as [a ends (R2) | b ends (R2)] (the
 * student's rows).  Deterministic integer work, 3 launches; oracle: pair_owner_assign. */
typedef struct llp_owner_cat {
  const int32_t* a; int64_t a_kc, a_kld, a_koff, a_kstep;
  const int32_t* b; int64_t b_kc, b_kld, b_koff, b_kstep;
  int32_t key_b; int32_t pad;
  int64_t n;
} llp_owner_cat;
int64_t llp_pair_owner_workspace_bytes(int64_t n0, int64_t n1, int64_t n2, int world);
int llp_pair_owner_assign(int ncat, const llp_owner_cat* cats, int64_t num_nodes, int world, int rank,
                          const int32_t* owner_tab, int32_t* sel, int32_t* gpos, int32_t* target, int64_t R2,
                          void* workspace, int64_t workspace_bytes, void* stream);
/* s_full[i] = s_loc[gpos[i] - lo] if lo <= gpos[i] < hi else 0 (i < n), t likewise (either
 * output may be NULL): this rank's context logits placed into the [B*C] grid that one SUM
 * all-reduce completes (the other ranks' slots are zero here). */
int llp_pair_owner_scatter(int64_t n, const int32_t* gpos, int64_t lo, int64_t hi, const float* s_loc,
                           const float* t_loc, float* s_full, float* t_full, void* stream);

/* out[r, :] = a[ia[r], :] * b[ib[r], :]   (ia/ib NULL = identity) — the
 * predictor input x_i * x_j (src/models.py:140) materialised once per step so
 * the first predictor layer's forward and weight-gradient GEMMs both stream it
 * with global_load_lds.  Rows of 16-byte multiples. */
int llp_hadamard_rows(int dtype, int64_t R, int64_t H, const void* a, const int32_t* ia, const void* b,
                      const int32_t* ib, void* out, void* stream);

/* ---------------------------------------------------------------- Hadamard backward
 * Backward of x_i * x_j (src/models.py:140) for the minibatch row layout of
 * src/main.py:95-105 (h rows: B anchor blocks of (1 + C) rows, then 2L src
 * rows, then 2L dst rows; predictor rows: B*C context pairs then 2L label
 * pairs).  Deterministic: every dh row is written exactly once.
 *   dh[anchor b]      = sum_c dZ[b*C+c] * h[ctx(b,c)]
 *   dh[ctx(b,c)]      = dZ[b*C+c] * h[anchor b]
 *   dh[src i]         = dZ[B*C+i] * h[dst i],  dh[dst i] = dZ[B*C+i] * h[src i]
 * hidx (may be NULL): h holds unique nodes only, target-layout row r reads h[hidx[r]]
 * (dh stays in the target layout). */
int llp_hadamard_bwd_blocks(int dtype, int64_t B, int64_t C, int64_t L2, int64_t H,
                            const void* dZ, const float* drow, const void* h, const int32_t* hidx, void* dh,
                            void* stream);

/* ---------------------------------------------------------------- unique-node compaction
 * The student MLP of train_minibatch runs on data.x[this_target] (src/main.py:95-96);
 * without dropout duplicate rows give identical activations, so the engine runs it
 * on the unique nodes.  llp_dedup_rows: uniq[0..U) = sorted distinct values of
 * target[0..R) (U -> *n_unique, device), pos[r] = slot of target[r]; seg_rows =
 * rows grouped by slot in row order (stable sort), seg_ptr[0..U] = group bounds.
 * llp_segment_sum_rows: out[u] = sum of src rows of group u (f32 accumulate,
 * fixed order: deterministic); out_rows (may be NULL): group u is written to
 * out row out_rows[u] (uniq: a scatter onto node rows, e.g. the teacher's
 * dh[N, H], src/train_teacher_gnn.py:62); u_dev (may be NULL): device count,
 * the call covers min(U, *u_dev) groups (grid sized by U: capturable);
 * out_dtype: dtype, or LLP_F32 for unrounded sums (bf16 input; a cross-rank
 * reduction follows, DistillEngine._fb_shard).
 * llp_gather_i32: out[i] = src[idx[i]]. */
int64_t llp_dedup_rows_workspace_bytes(int64_t num_nodes, int64_t R);
int llp_dedup_rows(int64_t num_nodes, int64_t R, const int32_t* target, int32_t* uniq, int32_t* pos,
                   int32_t* n_unique, int32_t* seg_ptr, int32_t* seg_rows, void* workspace,
                   int64_t workspace_bytes, void* stream);
/* llp_dedup_rows in four launches instead of ten (the same outputs): per-node counts, ONE
 * pass over the nodes (the exclusive scan by decoupled look-back between workgroups + the
 * compaction), the scatter, and every segment's sort in one launch.  The workspace
 * (llp_dedup_rows2_workspace_bytes) starts with llp_dedup_rows2_state_bytes(num_nodes) bytes
 * of state that persists between calls (counts, look-back flags tagged with a per-call
 * epoch, a ticket); state_clean = 1 vouches that they are as a previous llp_dedup_rows2 call
 * on this workspace (with this num_nodes) left them, or zero; 0 zeroes them first (one more
 * launch).  Word [2] of the 256-byte control block at the end of the state is set nonzero if
 * a look-back ever timed out (bounded spin; the results are then invalid).
 * zero_rows (may be NULL): rows [node * zero_ld_bytes, + zero_row_bytes) of the nodes absent
 * from target are zeroed in the same pass (16-B aligned multiples of 16 bytes) -- the
 * 'other rows are 0' of a per-node gradient scatter, without a fill of the whole matrix. */
int64_t llp_dedup_rows2_state_bytes(int64_t num_nodes);
int64_t llp_dedup_rows2_workspace_bytes(int64_t num_nodes, int64_t R);
int llp_dedup_rows2(int64_t num_nodes, int64_t R, const int32_t* target, int32_t* uniq, int32_t* pos,
                    int32_t* n_unique, int32_t* seg_ptr, int32_t* seg_rows, void* zero_rows,
                    int64_t zero_ld_bytes, int64_t zero_row_bytes, int state_clean, void* workspace,
                    int64_t workspace_bytes, void* stream);
int llp_segment_sum_rows(int dtype, int64_t U, int64_t H, const int32_t* seg_ptr, const int32_t* rows,
                         const void* src, int64_t ld_src, void* out, int64_t ld_out, int out_dtype,
                         const int32_t* out_rows, const int32_t* u_dev, void* stream);
int llp_gather_i32(int64_t n, const int32_t* idx, const int32_t* src, int32_t* out, void* stream);
/* out row r = src row idx[r] (row_bytes each; leading dimensions in bytes) for
 * r < min(n, *count_dev) (count_dev may be NULL): data.x[this_target]
 * (src/main.py:95) materialised once per step, so the first student layer's
 * forward and weight-gradient GEMMs read plain rows (the unique-node student:
 * idx = uniq, count_dev = n_unique). */
int llp_gather_rows(int64_t n, int64_t row_bytes, const int32_t* idx, const void* src, int64_t ld_src_bytes,
                    void* out, int64_t ld_out_bytes, const int32_t* count_dev, void* stream);
/* Backward of the predictor input h[i] * h[j] (src/main.py:102-103,126) reduced
 * straight onto the unique nodes, bit-identical to llp_hadamard_bwd_blocks (hidx =
 * pos) followed by llp_segment_sum_rows: dh[u] = sum over the target rows of node u
 * (seg_ptr / rows from llp_dedup_rows, row order) of each row's Hadamard gradient
 * as the row kernel would store it, f32 accumulation, one write per node, without
 * the [R1, H] row buffer.  anchor_rows: caller-owned [B, H] scratch (compute dtype)
 * for the anchors' context sums.  Row layouts as llp_hadamard_bwd_blocks; h is the
 * unique-node table [U, H], pos maps target rows to it; drow (dZ = NULL) is the
 * 'inner' predictor's per-pair scalar.  dh rows are of out_dtype (dtype, or LLP_F32:
 * the sums unrounded, for a following cross-rank reduction) and node u's sum goes to
 * row out_rows[u] (NULL: row u).  With B = C = 0 the rows are the label-row layout
 * alone: the full-batch student's d(h[ia] * h[ib]) with pos = [ia | ib] node ids, h
 * the [N, H] node table and out_rows = the unique node ids (src/main.py:173-235). */
int llp_hadamard_bwd_segments(int dtype, int64_t U, int64_t B, int64_t C, int64_t L2, int64_t H,
                              const int32_t* seg_ptr, const int32_t* rows, const int32_t* pos, const void* dZ,
                              const float* drow, const void* h, void* anchor_rows, void* dh, int64_t ld_dh,
                              int out_dtype, const int32_t* out_rows, const int32_t* u_dev, void* stream);

/* Generic scatter form (full-batch train(), src/main.py:173-214, where rows of
 * h repeat): dh[ia[r]] += dZ[r]*h2[ib[r]],  dh[ib[r]] += dZ[r]*h1[ia[r]]
 * with f32 atomics into dh (f32).  For both forms drow != NULL replaces dZ by
 * the row-broadcast dZ[r, :] = drow[r] (the 'inner' predictor, src/models.py:147-148). */
int llp_hadamard_bwd_scatter(int dtype, int64_t R, int64_t H, const void* dZ, const float* drow,
                             const int32_t* ia, const int32_t* ib, const void* h, float* dh, void* stream);

/* ---------------------------------------------------------------- samplers
 * Context sampler, src/main.py:33-50 + torch_cluster random_walk (p=q=1,
 * coalesced=False semantics: rowptr = degree-count prefix sum of `row`,
 * neighbours = col[rowptr[n]:rowptr[n+1]] in the given order).
 * samples[b, 0] = start[b]; then the walks (ps_method 0 = 'rw': one walk of
 * rw_step*hops steps; 1 = 'nb': rw_step walks of `hops` steps, start column
 * dropped after the first); then rw_step*hops*ns_rate uniform negatives.
 * Philox stream of walk i = stream_base + i, negatives stream_base + rw_step,
 * with stream_base = 64*(*step_ctr) + stream_offset (device counter: graph-safe).
 * Draw indices use the GLOBAL anchor position b + b_offset, so a rank holding
 * anchors [b_offset, b_offset + B) draws what a single GPU would. */
int llp_context_sampler(const int32_t* rowptr, const int32_t* col, int64_t num_nodes,
                        const int32_t* start, int64_t B, int64_t b_offset, int ps_method, int rw_step,
                        int hops, int ns_rate, uint64_t seed, const int64_t* step_ctr,
                        int64_t stream_offset, int32_t* samples, void* stream);

/* torch.randint(0, N, [2, n_total]) (src/main.py:84,209) restricted to columns
 * [offset, offset + n): out[0..n) = row 0, out[n..2n) = row 1.  Philox stream
 * 64*(*step_ctr) + stream_offset, draw #(row*n_total + column). */
int llp_randint_pairs(int64_t num_nodes, int64_t n, int64_t n_total, int64_t offset, uint64_t seed,
                      const int64_t* step_ctr, int64_t stream_offset, int32_t* out, void* stream);

/* The step's batch of two epoch permutations, read on the device so a replayed hipGraph
 * feeds itself (DataLoader(range(E), P, shuffle=True) / node_perm slices, src/main.py:72-73,
 * 168-170): out_a[i] = perm_a[j*stride_a + off_a + i] (i < n_a), out_b likewise, with
 * j = (*step_ctr + ctr_offset) mod n_batches.  len_a / len_b: the permutations' lengths
 * (every j < n_batches must stay inside them). */
int llp_batch_slices(const int32_t* perm_a, int64_t stride_a, int64_t off_a, int64_t n_a,
                     const int32_t* perm_b, int64_t stride_b, int64_t off_b, int64_t n_b,
                     int64_t n_batches, int64_t len_a, int64_t len_b, const int64_t* step_ctr,
                     int64_t ctr_offset, int32_t* out_a, int32_t* out_b, void* stream);

/* Per-step index build for the minibatch layout (src/main.py:78,81-95):
 * pos edges = pairs[perm[*step_ctr*P_stride + i]] (i < P), neg edges =
 * neg[2, ld_neg] columns [0, n_neg) (randint: n_neg = P; PyG dense: may be fewer);
 * target (node id per h row) = [samples.flatten(), src(P+n_neg), dst(P+n_neg)]. */
int llp_build_targets(int64_t B, int64_t C1, const int32_t* samples, const int32_t* pairs,
                      const int32_t* perm, const int64_t* step_ctr, int64_t perm_stride,
                      int64_t P, const int32_t* neg, int64_t n_neg, int64_t ld_neg, int32_t* target,
                      void* stream);

/* Teacher / predictor pair indices from samples: ia[b*C+c] = samples[b,0],
 * ib[b*C+c] = samples[b,1+c]  (src/main.py:104,106). */
int llp_pair_index_from_samples(int64_t B, int64_t C, const int32_t* samples,
                                int32_t* ia, int32_t* ib, void* stream);

/* One minibatch step's index building in ONE launch (the collab path of
 * train_minibatch: neighbor_samplers src/main.py:33-50 + torch.randint negatives
 * :83-84 + this_target :95 + the teacher's pair index :104,106): exactly
 * llp_context_sampler(.., stream_offset, samples) + llp_randint_pairs(num_nodes, P,
 * P_total, p_offset, seed, step_ctr, neg_stream_offset, neg) + llp_build_targets(B,
 * C1, samples, pairs, perm, NULL, 0, P, neg, P, P, target) +
 * llp_pair_index_from_samples(B, C, samples, t_ia, t_ib), same draws, bit for bit (t_ia = t_ib =
 * NULL skips the pair index: the owner decomposition builds its own). */
int llp_minibatch_sample(const int32_t* rowptr, const int32_t* col, int64_t num_nodes, const int32_t* start,
                         int64_t B, int64_t b_offset, int ps_method, int rw_step, int hops, int ns_rate,
                         uint64_t seed, const int64_t* step_ctr, int64_t stream_offset, const int32_t* pairs,
                         const int32_t* perm, int64_t P, int64_t P_total, int64_t p_offset,
                         int64_t neg_stream_offset, int32_t* samples, int32_t* neg, int32_t* target,
                         int32_t* t_ia, int32_t* t_ib, void* stream);

/* ---------------------------------------------------------------- full-batch step (src/main.py:147-236)
 * Dense negative sampling, replacing PyG 2.2.0 negative_sampling(edge_index,
 * num_nodes, num_neg_samples, method='dense') (src/main.py:206,
 * src/train_teacher_gnn.py:50).  edge_keys: sorted unique int64 keys
 * row*(N-1) + col - (row < col) of the non-self-loop edges.  sample_size =
 * int(1.1*num_neg/prob) as PyG computes it (host, with duplicate edges counted).
 * edge_table (may be NULL): the keys' set from llp_edge_table_build, used instead of
 * the sorted edge_keys for the membership test.
 * population = N(N-1) <= sample_size: the non-edges in ascending order (bit-exact
 * with PyG).  Otherwise `rounds` * sample_size Philox candidates (stream
 * 64*(*step_ctr)+stream_offset), duplicates and existing edges dropped, first
 * num_neg kept in draw order — the law of PyG's sample-without-replacement
 * rounds.  out = int32[2, ld_out] (row 0 = source); *count = columns written
 * (may be < num_neg, as PyG's may). */
int64_t llp_neg_sample_dense_workspace_bytes(int64_t max_candidates);
int llp_neg_sample_dense(int64_t num_nodes, const int64_t* edge_keys, int64_t n_keys,
                         const uint64_t* edge_table, int64_t edge_table_size, int64_t num_neg,
                         int64_t sample_size, int rounds, uint64_t seed, const int64_t* step_ctr,
                         int64_t stream_offset, int32_t* out, int64_t ld_out, int32_t* count,
                         void* workspace, int64_t workspace_bytes, void* stream);
/* llp_neg_sample_dense in two launches (the same outputs): the candidates, then ONE pass
 * that counts, scans (decoupled look-back over tiles) and scatters.  The candidates' set and
 * the look-back flags persist in the workspace (llp_neg_sample_dense2_workspace_bytes,
 * its first llp_neg_sample_dense2_state_bytes bytes) tagged with a per-call epoch instead of
 * being cleared each call; state_clean = 1 vouches that a previous call with the same
 * max_candidates left them (or that they are zero), 0 clears them first (one more launch).
 * Needs N(N-1) < 2^40. */
int64_t llp_neg_sample_dense2_state_bytes(int64_t max_candidates);
int64_t llp_neg_sample_dense2_workspace_bytes(int64_t max_candidates);
int llp_neg_sample_dense2(int64_t num_nodes, const int64_t* edge_keys, int64_t n_keys,
                          const uint64_t* edge_table, int64_t edge_table_size, int64_t num_neg,
                          int64_t sample_size, int rounds, uint64_t seed, const int64_t* step_ctr,
                          int64_t stream_offset, int32_t* out, int64_t ld_out, int32_t* count,
                          int state_clean, void* workspace, int64_t workspace_bytes, void* stream);
/* The graph's edge keys (PyG's dense encoding, as edge_keys above) in an open-addressing
 * set of llp_edge_table_size(n_keys) slots (a power of two), built once per graph; passed
 * to llp_neg_sample_dense as edge_table (edge_keys may then be NULL), a candidate's
 * membership test is one or two probes instead of a binary search of the sorted keys.
 * Same results either way. */
int64_t llp_edge_table_size(int64_t n_keys);
int llp_edge_table_build(const int64_t* edge_keys, int64_t n_keys, uint64_t* table, int64_t table_size,
                         void* stream);

/* Predictor-row indices of the full-batch step: rows [0, B*C) are (anchor,
 * context) pairs from samples[B, C1] (src/main.py:184-186), then P positives
 * pairs[perm[i]] and n_neg negatives neg[:, i] (train_edges, src/main.py:212).
 * neg_count (may be NULL): negative slot i is live while neg_offset + i < *neg_count
 * (llp_llp_loss); later slots become the inert pair (0, 0). */
int llp_fullbatch_pairs(int64_t B, int64_t C1, const int32_t* samples, const int32_t* pairs,
                        const int32_t* perm, int64_t P, const int32_t* neg, int64_t ld_neg, int64_t n_neg,
                        const int32_t* neg_count, int64_t neg_offset, int32_t* ia, int32_t* ib, void* stream);

/* KD terms of the full-batch loss (src/main.py:218-219):
 *   KD_LM = mse(sigmoid(out_logit), t_prob_lab)  over n_lab rows (normaliser n_lab_total);
 *           dlogit_lab += loss_scale * w_lm * d/dlogit
 *   KD_RM = 1 - mean_b cos(h[idx_rm[b]], t_h[idx_rm[b]])  (src/main.py:24-25; normaliser
 *           B_rm_total); dh[idx_rm[b]] += loss_scale * w_rm * d/dh  (dh f32, may be NULL)
 * terms_out[4] = KD_RM share, terms_out[5] = KD_LM share, terms_out[0] += weighted sum. */
int64_t llp_kd_terms_workspace_bytes(int64_t B_rm, int64_t n_lab);
int llp_kd_terms(int dtype, int64_t n_lab, const float* out_logit, const float* t_prob_lab,
                 double n_lab_total, float w_lm, int64_t B_rm, int64_t H, const void* h, int64_t ldh,
                 const void* t_h, int64_t ldt, const int32_t* idx_rm, double B_rm_total, float w_rm,
                 float loss_scale, float* dlogit_lab, float* dh, int64_t lddh, float* terms_out,
                 void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- evaluation (src/train_teacher_gnn.py:76-268)
 * Hits@K as ogb 1.3.6 Evaluator computes it (src/train_teacher_gnn.py:121-143,
 * 227-247): kth = topk(neg, K)[-1] (exact radix select), hits = #(pos > kth) /
 * n_pos; n_neg < K -> 1.0.  One result per entry of Ks[n_K] (device int32). */
int llp_hits_at_k(const float* pos, int64_t n_pos, const float* neg, int64_t n_neg, const int32_t* Ks,
                  int n_K, double* hits_out, void* stream);
/* sklearn roc_auc_score(y, score) with y = [1]*n_pos + [0]*n_neg
 * (src/train_teacher_gnn.py:153,263): Mann-Whitney U / (n_pos*n_neg), ties 1/2. */
int64_t llp_auc_workspace_bytes(int64_t n_pos, int64_t n_neg);
int llp_auc(const float* pos, int64_t n_pos, const float* neg, int64_t n_neg, double* auc_out,
            void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- SAGE aggregate
 * out[i] = scale_i * sum_{e in [rowptr[i], rowptr[i+1])} w_e * x[col[e]]
 *   mode 0 (forward mean):   scale_i = 1/max(deg_i,1), w_e = 1
 *   mode 1 (backward of mean over the transposed CSR): scale_i = 1,
 *          w_e = inv_deg[col[e]]
 * PyG MessagePassing(aggr='mean') as used by SAGEConv / SAGEConv_updated
 * (src/models.py:113, src/sageconv_updated.py:71-72), duplicates counted (Q2). */
int llp_csr_aggregate(int dtype, int64_t n_rows, int64_t F, const int32_t* rowptr, const int32_t* col,
                      const void* x, int64_t ldx, const float* inv_deg, int mode,
                      void* out, int64_t ldo, int accumulate, void* stream);

/* GCN propagation, replaces torch_geometric 2.2.0 GCNConv.propagate after
 * gcn_norm (GCNConv(cached=True) at src/models.py:60-64, GCN.forward :72-78):
 *   out[i] = dinv[i] * sum_{e in row i} dinv[col[e]] * x[col[e]]  (+ bias)
 * over the CSR-by-destination of the graph with its self-loops replaced by
 * one loop per node (dinv = deg^-1/2 of that graph).  Over the transposed CSR
 * with bias = NULL it is the backward dX of the same propagation. */
int llp_gcn_aggregate(int dtype, int64_t n_rows, int64_t F, const int32_t* rowptr, const int32_t* col,
                      const void* x, int64_t ldx, const float* dinv, const float* bias, void* out, int64_t ldo,
                      int accumulate, void* stream);

/* ---------------------------------------------------------------- optimiser tail
 * Multi-tensor clip_grad_norm_(group, max_norm) per group (Q9) + Adam
 * (torch.optim.Adam defaults, src/main.py:134-138,400-402).  Descriptor tables
 * live in device memory (static per engine): see llp_tensor_desc. */
typedef struct llp_tensor_desc {
  float* param;        /* f32 master weights                                     */
  float* grad;         /* f32 gradient                                           */
  float* exp_avg;
  float* exp_avg_sq;
  void* shadow;        /* optional copy of param (same shape), or NULL           */
  void* shadow_t;      /* optional transposed copy [cols][rows], or NULL         */
  int64_t numel;
  int64_t rows;        /* for the transposed copy                                */
  int64_t cols;
  int32_t group;       /* clip group id (0..7)                                   */
  int32_t shadow_dtype;/* element type of shadow / shadow_t: LLP_F32 or LLP_BF16 */
  int64_t shadow_ld;   /* row stride of shadow (0 = cols): lets two parameters share one
                          K-concatenated GEMM operand, e.g. [W_l | W_r] of a SAGEConv  */
  int64_t shadow_t_ld; /* row stride of shadow_t (0 = rows)                            */
} llp_tensor_desc;

/* sumsq[g] = sum of grad^2 over tensors of group g (n_groups <= 8). */
int64_t llp_grad_sumsq_workspace_bytes(int n_tensors, int64_t max_numel);
int llp_grad_sumsq(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int n_groups,
                   float* sumsq, void* workspace, int64_t workspace_bytes, void* stream);
/* clip coef per group = min(1, max_norm/(sqrt(sumsq)+1e-6)) applied to the
 * grads in place (as clip_grad_norm_ does); Adam step number *step (device,
 * incremented by this call); refreshes the shadows.  sumsq NULL = no clip. */
int llp_adam_step(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, const float* sumsq,
                  float max_norm, float lr, float beta1, float beta2, float eps, int64_t* step,
                  void* stream);
/* The same two calls in ONE launch each.  llp_grad_sumsq_t (ticket: a ticket block of
 * LLP_TICKET_WORDS; NULL = the two-launch form): the finalize runs in the last workgroup to
 * arrive.  llp_adam_step_t: Adam writes both shadows in its own pass (transposed ones through
 * 32 x 32 LDS tiles) and reads *step WITHOUT advancing it: the caller advances it after the
 * launch (llp_step_end2).  Results bit-identical to the two-launch forms. */
int llp_grad_sumsq_t(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int n_groups,
                     float* sumsq, uint32_t* ticket, void* workspace, int64_t workspace_bytes, void* stream);
int llp_adam_step_t(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, const float* sumsq,
                    float max_norm, float lr, float beta1, float beta2, float eps, const int64_t* step,
                    void* stream);
/* The one-launch forms on a COMPACT 1-D grid of n_work workgroups, one work item each (round 5):
 * n_work = the sum over the table of llp_grad_sumsq_work_items(numel) (gradient norm) or of
 * llp_adam_work_items(numel, rows, cols, shadow_t != NULL) (Adam), which the caller computes
 * once from its tensors' shapes.  The 2-D grids of llp_grad_sumsq_t / llp_adam_step_t (max chunks
 * x tensors) leave most workgroups idle past the small tensors' ends, and each idle one still
 * loads its descriptor: ~20k in the coauthor-physics optimizer.  Same arithmetic, same order:
 * bit-identical results.  llp_grad_sumsq_w requires the ticket block. */
int64_t llp_grad_sumsq_work_items(int64_t numel);
int64_t llp_adam_work_items(int64_t numel, int64_t rows, int64_t cols, int transposed_shadow);
int llp_grad_sumsq_w(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int64_t n_work, int n_groups,
                     float* sumsq, uint32_t* ticket, void* workspace, int64_t workspace_bytes, void* stream);
int llp_adam_step_w(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, int64_t n_work,
                    const float* sumsq,
                    float max_norm, float lr, float beta1, float beta2, float eps, const int64_t* step,
                    void* stream);
/* Refresh bf16 shadows from masters (after loading weights). */
int llp_refresh_shadows(const llp_tensor_desc* descs, int n_tensors, int64_t max_numel, void* stream);

/* ---------------------------------------------------------------- small utilities */
int llp_convert(int src_dtype, int dst_dtype, int64_t n, const void* src, void* dst, void* stream);
/* Sum loss terms into a running total (device), so an epoch needs one host sync. */
int llp_accumulate(int64_t n, const float* src, float weight, double* dst, void* stream);
int llp_increment(int64_t* ctr, void* stream);
/* The end of a training step in one launch: *loss_sum += (double)*loss * weight (the
 * epoch's total_loss += loss.item() * num_examples, src/main.py:140-141) and
 * *step_ctr += 1 (the device step counter that keys every Philox stream). */
int llp_step_end(const float* loss, float weight, double* loss_sum, int64_t* step_ctr, void* stream);
/* llp_step_end that also advances the Adam step counter *adam_step (after llp_adam_step_t). */
int llp_step_end2(const float* loss, float weight, double* loss_sum, int64_t* step_ctr, int64_t* adam_step,
                  void* stream);
/* Zero `bytes` bytes at p by a kernel (no memset node: a captured hipMemsetAsync node
 * was measured not to do its work on replay). */
int llp_zero(void* p, int64_t bytes, void* stream);

/* Elementwise pieces of the module-level autograd ops (models.py):
 * out = alpha * gy * (y > 0)   (y NULL: no mask)  — ReLU/dropout backward (src/models.py:52-53)
 * dst[c, r] = src[r, c]                           — weight transpose for data-gradients
 * out = a * b                                     — x_i * x_j backward (src/models.py:140)
 * out[r, :] = z[r, :] * s[r]                      — 'inner' predictor backward
 * out = gprob * prob * (1 - prob)                 — torch.sigmoid backward (src/models.py:150) */
int llp_relu_bwd(int dtype, int64_t n, const void* gy, const void* y, float alpha, void* out, void* stream);
/* Strided [rows, cols] forms for the SAGE teacher's concatenated layouts:
 * y = dropout(act(x)) (act NONE/RELU; dropout keep draw of (r, c), as the GEMM
 * epilogue; src/models.py:117-118) and out = alpha * gy * (y > 0). */
int llp_act_2d(int dtype, int64_t rows, int64_t cols, const void* x, int64_t ldx, void* y, int64_t ldy,
               int act, const llp_dropout* dropout, void* stream);
int llp_relu_bwd_2d(int dtype, int64_t rows, int64_t cols, const void* gy, int64_t ldg, const void* y,
                    int64_t ldy, float alpha, void* out, int64_t ldo, void* stream);
int llp_transpose(int dtype, int64_t rows, int64_t cols, const void* src, void* dst, void* stream);
int llp_mul(int dtype, int64_t n, const void* a, const void* b, void* out, void* stream);
int llp_row_scale(int dtype, int64_t rows, int64_t cols, const void* z, const float* s, void* out, void* stream);
int llp_sigmoid_bwd(int64_t n, const float* gprob, const float* prob, float* out, void* stream);

/* ---------------------------------------------------------------- norm_type
 * nn.LayerNorm(H) / nn.BatchNorm1d(H) after a hidden layer, fused with the ReLU and
 * dropout that follow it: MLP.forward src/models.py:45-54 (norms built at :27-37),
 * SAGE.forward src/models.py:110-119 (:90-101).  y = the layer's pre-norm output
 * [M, H], out = dropout(relu(norm(y))) [M, H] (relu 0: no ReLU), leading dimensions
 * ldy / ldo.  stats (f32): mean and 1/sqrt(var + eps), LayerNorm [2][M] per row,
 * BatchNorm [2][H] per column.  m_dev: optional device row count (LayerNorm only:
 * rows past it are not touched).  Dropout draw #(r*H + c) of the layer's stream, as
 * the GEMM epilogue.  Column sums are f64 [2][H], reduced in a fixed order
 * (deterministic); a batch split over ranks SUM-all-reduces them between the sum call
 * and the call that consumes them, and then normalises as the whole batch would. */
enum llp_norm_kind { LLP_NORM_LAYER = 1, LLP_NORM_BATCH = 2 };
int64_t llp_norm_workspace_bytes(int64_t M, int64_t H);
/* BatchNorm statistics: sums[0:H] = sum_r y[r, :], sums[H:2H] = sum_r y[r, :]^2. */
int llp_norm_colsums(int dtype, int64_t M, int64_t H, const void* y, int64_t ldy, const int32_t* m_dev,
                     double* sums, void* ws, void* stream);
/* Forward.  LayerNorm: per-row statistics into stats.  BatchNorm, training: mean and
 * biased variance from sums over `count` rows, running_mean / running_var updated with
 * `momentum` (unbiased variance) and *num_batches_tracked += 1, as torch's
 * BatchNorm1d.train(); eval: the running statistics (sums unused). */
int llp_norm_fwd(int kind, int dtype, int64_t M, int64_t H, const void* y, int64_t ldy, const float* gamma,
                 const float* beta, float eps, int training, const double* sums, double count, float momentum,
                 float* running_mean, float* running_var, int64_t* num_batches_tracked, float* stats,
                 const int32_t* m_dev, int relu, const llp_dropout* dropout, void* out, int64_t ldo, void* stream);
/* Backward, step 1: g = alpha * gout * (out > 0) (out NULL: no mask), xhat the
 * normalised y; sums[0:H] = sum_r g, sums[H:2H] = sum_r g * xhat, also written as
 * dbeta / dgamma (f32, may be NULL) -- this call's rows' share of them. */
int llp_norm_bwd_sums(int kind, int dtype, int64_t M, int64_t H, const void* gout, int64_t ldg, const void* out,
                      int64_t ldo, float alpha, const void* y, int64_t ldy, const float* stats, const int32_t* m_dev,
                      double* sums, float* dgamma, float* dbeta, void* ws, void* stream);
/* Backward, step 2: gy = d(loss)/dy.  LayerNorm: rstd * (a - mean_c(a) - xhat * mean_c(a * xhat)),
 * a = gamma * g, per row (sums unused); BatchNorm (training statistics):
 * gamma * rstd * (g - sums[c] / count - xhat * sums[H + c] / count). */
int llp_norm_bwd(int kind, int dtype, int64_t M, int64_t H, const void* gout, int64_t ldg, const void* out,
                 int64_t ldo, float alpha, const void* y, int64_t ldy, const float* gamma, const float* stats,
                 const double* sums, double count, const int32_t* m_dev, void* gy, int64_t ldgy, void* stream);

/* ---------------------------------------------------------------- diagnostics
 * Practical bf16 MFMA ceiling (bench.py roofline.practical_peak): one 512-thread
 * workgroup per CU issues v_mfma_f32_16x16x32_bf16 back to back on register operands
 * taken from `data` (n_u4 16-byte chunks of random bf16), `iters` iterations of 16
 * MFMAs over 4 x 4 operand pairs into 8 accumulators per wave; *flops = the FLOP count
 * of the launch (host);
 * out (llp_mfma_probe_out_floats() floats) keeps the accumulators live. */
int llp_mfma_probe(const void* data, int64_t n_u4, int64_t iters, float* out, double* flops, void* stream);
/* The same loop on v_mfma_f32_16x16x4_f32 (the fp32 GEMMs' instruction) over n random f32. */
int llp_mfma_probe_f32(const float* data, int64_t n, int64_t iters, float* out, double* flops, void* stream);
int64_t llp_mfma_probe_out_floats(void);
/* Diagnostics of round 6, not used by the engines:
 * llp_stage_probe: one wave per SIMD issuing v_mfma_f32_32x32x16_bf16 back to back beside `pieces`
 *   (0 / 4 / 8 / 16 per 32 MFMAs) operand-staging pieces of kind `mode` (0 none, 1 LDS-DMA, 2 global
 *   load into VGPRs + ds_write, 3 ds_read), reading src (src_u4 16-B chunks, src_u4 / 64 a power of
 *   two); per-workgroup shader cycles into cycles[], accumulators into out.
 * llp_gemm_nt_w4_probe: the one-wave-per-SIMD persistent NT GEMM (csrc/gemm256_w4.hip), bf16,
 *   N % 256 == 0, K % 128 == 0; act 0 plain / 1 ReLU (+ bit mask out) / 3 ReLU backward through
 *   mask_in; diag selects the diagnostic builds' skips (0: the whole kernel).  Bit-identical to
 *   llp_gemm_nt where both run. */
int llp_stage_probe(int mode, int pieces, const void* src, int64_t src_u4, int64_t iters, float* out,
                    unsigned long long* cycles, void* stream);
int llp_gemm_nt_w4_probe(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                         void* C, int64_t ldc, const float* bias, int act, float alpha, void* mask_out,
                         const void* mask_in, int64_t ld_mask, int diag, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LLP_HIP_H_ */
