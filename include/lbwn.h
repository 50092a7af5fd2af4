/* lbwn — MI355X-native WaveNet hot path, C ABI.
 *
 * Drop-in boundary for hrbigelow/lb-wavenet's TensorFlow graph builders.  The reference
 * has no FFI (it is pure Python over TensorFlow 1.x C++ kernels); each entry point below
 * replaces the TF kernel sequence built at the cited reference line.  Host code (the
 * Python `lbwn` package, or any C/C++ caller) owns every buffer; the library never
 * allocates device memory, never synchronises, and is stateless except for the opaque
 * plan (shapes + workspace carving).  All device pointers are fp32 [B][T][C]
 * channels-last unless noted; int32 for µ-law codes and voice ids.  Every call is
 * stream-ordered on the caller's hipStream_t (passed as void*; NULL = default stream).
 * Return value: 0 on success, otherwise a hipError_t or 22 (EINVAL); the message is
 * available from lbwn_last_error() (thread-local).  Errors mirror the reference's
 * "print to stderr + exit(1)" checks (arch.py:147-161) as return codes instead.
 */
#ifndef LBWN_H
#define LBWN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBWN_ABI_VERSION 2

/* par/arch*.json after normalisation (tmodel.py:10-23, arch.py:31-103). */
typedef struct lbwn_arch {
  int n_blocks, n_block_layers;
  int n_quant, n_res, n_dil, n_skip, n_post;
  int n_gc_embed, n_gc_category; /* n_gc_embed == 0: no global conditioning */
  int n_lc_in, n_lc_out;         /* n_lc_out == 0: no local conditioning     */
  int n_lc_upsample;
  int lc_upsample[8];
  int use_bias;
} lbwn_arch;

/* Device pointers into a caller-owned flat fp32 buffer, reference layouts
 * (arch.py:85-103).  Per-layer tensors of one kind are contiguous over the
 * L = n_blocks*n_block_layers layers in (block, layer) order, e.g. sig = SIGNAL_0_0,
 * SIGNAL_0_1, ... each [2][n_res][n_dil].  Bias pointers are NULL when !use_bias; GC/LC
 * pointers are NULL when the arch has no GC/LC. */
typedef struct lbwn_params {
  float* pre;   float* pre_b;          /* PRE [Q][Cr], PRE_BIAS [Cr]                    */
  float* sig;   float* sig_b;          /* SIGNAL [L][2][Cr][Cd], SIGNAL_BIAS [L][Cd]     */
  float* gate;  float* gate_b;         /* GATE   [L][2][Cr][Cd], GATE_BIAS   [L][Cd]     */
  float* res;   float* res_b;          /* RESIDUAL [L][Cd][Cr], RESIDUAL_BIAS [L][Cr]    */
  float* skip;  float* skip_b;         /* SKIP [L][Cd][Cs], SKIP_BIAS [L][Cs]            */
  float* gc_embed;                     /* GC_EMBED [n_cat+1][Ge]                         */
  float* gc_sig; float* gc_gate;       /* GC_SIGNAL/GC_GATE [L][Ge][Cd]                  */
  float* lc_sig; float* lc_gate;       /* LC_SIGNAL/LC_GATE [L][Clc][Cd]                 */
  float* lc_up[8];                     /* LC_UPSAMPLE_i [s_i][Clc][dim2]                 */
  float* post1; float* post1_b;        /* POST1 [Cs][Cp], POST1_BIAS [Cp]                */
  float* post2; float* post2_b;        /* POST2 [Cp][Q],  POST2_BIAS [Q]                 */
} lbwn_params;

const char* lbwn_last_error(void);
int lbwn_abi_version(void);

/* ---- plan: the WaveNetTrain graph for a fixed (arch, batch_sz, slice_sz) ------------ */
typedef struct lbwn_plan lbwn_plan;
/* replaces WaveNetTrain.__init__ + build() graph construction (tmodel.py:8-48, :292-340) */
int lbwn_plan_create(const lbwn_arch* arch, int batch_sz, int slice_sz, lbwn_plan** out);
void lbwn_plan_destroy(lbwn_plan* plan);
size_t lbwn_plan_workspace_bytes(const lbwn_plan* plan);
/* Byte offset/size of a named workspace tensor (for parity tests / debugging):
 * "x" [L][B][H+T][n_res] (layer inputs with D-sep halo, H = 2^(n_block_layers-1)),
 * "z" [M][L·n_dil] (gate outputs), "s" [M][n_skip] (skip sum), "r2" [M][n_post],
 * "logits" [M][n_quant] (dlogits after forward), "dh" [M][n_post], "ds" [M][n_skip],
 * "dz" [M][L·n_dil] (backward; with the bf16-split chains in the chain's 32-row block order
 * instead of rows), "status" (int32: 0, or the code of a chain hand-off that timed out), and
 * for conditioned archs "cond" [M][L·2·n_dil] (LC term), "dvall" (its dv: rows [M][L·2·n_dil],
 * or after a bf16-split chain backward k-blocked [2L][ceil(M/32)·32][32], the size reported
 * accordingly), "gctab"/"gcd" [n_cat+1][L·2·n_dil] (GC table, its gradient).  */
int lbwn_plan_tensor(const lbwn_plan* plan, const char* name, size_t* offset, size_t* bytes);
/* One-shot timing probe: the next lbwn_train_forward/backward on this plan records
 * hipEvent_t ev_start right before and ev_stop right after the named launch(es):
 * "layer_fwd" (the residual stack: the persistent chain launch, or the span of the
 * per-layer launches; "layer_fwd@<l>" = layer l of the per-layer path), "layer_bwd",
 * "layer_reduce", "skip_fwd" (S = Zcat·SKIPcat), "post1_fwd", "post2_fwd", "head", "lc_cond",
 * "dpost2", "dh", "dpost1", "ds", "dskip" (Zcatᵀ·dS), "dz" (dS·SKIPcatᵀ).  Events are the
 * caller's (e.g. torch.cuda.Event(enable_timing=True).cuda_event). */
int lbwn_plan_probe(lbwn_plan* plan, const char* launch_name, void* ev_start, void* ev_stop);
/* Make `stream` wait (hipStreamWaitEvent, no host sync) for a point of the last
 * lbwn_train_backward on this plan, so that a data-parallel caller can start a gradient
 * all-reduce bucket before the backward ends.  point "head_grads": the POST1/POST2 weight
 * gradients, their biases and SKIP_BIAS are final and the backward chain has completed (no
 * collective can then share the chip with a persistent chain launch).  point "side_grads": the
 * end of the plan's side stream -- PRE, SIGNAL, GATE, RESIDUAL, the GC tables and their biases
 * are final (dSKIP may still run).  *waited = 1 if the plan has that point (chain plans; for
 * "head_grads" without padded head widths), else 0 and nothing is enqueued (wait for the whole
 * backward instead).  Added in ABI 2 ("side_grads": round 6, same ABI). */
int lbwn_plan_stream_wait(lbwn_plan* plan, const char* point, void* stream, int* waited);
/* receptive field F = n_blocks·Σ2^l (tmodel.py:50-51) */
int lbwn_recep_field_sz(const lbwn_arch* arch);

/* Forward + loss of one slice (tmodel.py:292-328 + _loss_fcn :218-289).
 *   wav_q  int32 [B][T] µ-law codes; ids int32 [B][T] (0 = invalid window);
 *   mel    fp32 [B][T/hop][n_lc_in] or NULL;  save fp32 D-sep state, layers packed in
 *          (block, layer) order, each SAVE_{d}_{b}_{bl} [B][d][n_res]; read (prepend) and
 *          updated in place (tmodel.py:122-127, :163-166).
 *   stats  fp32[4] out: Σ masked xent, n_valid, Σ|argmax diff|·mask, 1/n_valid (0 if none).
 * The plan's workspace keeps the activations for lbwn_train_backward. */
int lbwn_train_forward(lbwn_plan* plan, const lbwn_params* params, void* workspace, const int* wav_q,
                       const int* ids, const float* mel, float* save, float* stats, void* stream);

/* Gradients of Σ masked xent (NOT divided by n_valid, no l2 term: both are applied in
 * lbwn_adam_tf1, so data-parallel ranks can all-reduce raw sums).  Replaces
 * compute_gradients (tmodel.py:354-358).  Must follow lbwn_train_forward on the same
 * workspace/stream.  grads: every pointer of the struct is fully overwritten. */
int lbwn_train_backward(lbwn_plan* plan, const lbwn_params* params, const lbwn_params* grads, void* workspace,
                        const int* wav_q, const int* ids, const float* mel, void* stream);

/* tf.train.AdamOptimizer.apply_gradients (train.py:178, :186), TF1 semantics, over the
 * flat buffers [0, n_total); elements [0, n_weights) are non-BIAS trainables and get the
 * l2 term (tmodel.py:250-261): g = raw·inv_n + l2_factor·θ with inv_n = 1/stats[1]
 * (0 if stats[1] == 0).  counters int64[4]: [0] GLOBAL_STEP, [1] VALID_SAMPLES,
 * [2] Adam applies so far (t-1), [3] cumulative status (every step's status word ORed in,
 * never reset by a step).  lr_t = lr·√(1-β2^t)/(1-β1^t) is derived on device, so the call
 * is graph-capturable.  Then counters advance by (1, n_valid, 1).
 * step_status (nullable): the plan's "status" word of this step (under data parallelism the
 * sum over ranks).  Nonzero means a chain hand-off timed out and the gradients are garbage:
 * the update is skipped on the device (params, m, v and counters[0..2] unchanged) and the
 * word is ORed into counters[3], so the host needs no per-step synchronisation.
 * (ABI 2: step_status added.) */
int lbwn_adam_tf1(float* params, const float* grads, float* m, float* v, int64_t n_weights, int64_t n_total,
                  float lr, float beta1, float beta2, float eps, float l2_factor, const float* stats,
                  int64_t* counters, const uint32_t* step_status, void* stream);

/* ---- cached autoregressive generation (imodel.WaveNetGen, imodel.py:7-303) ------------ */
typedef struct lbwn_gen_plan lbwn_gen_plan;
/* B streams, outputs for up to max_steps samples, teacher vector up to max_teacher codes. */
int lbwn_gen_plan_create(const lbwn_arch* arch, int batch_sz, int64_t max_steps, int64_t max_teacher,
                         lbwn_gen_plan** out);
void lbwn_gen_plan_destroy(lbwn_gen_plan* plan);
size_t lbwn_gen_workspace_bytes(const lbwn_gen_plan* plan);
/* "samples" int32 [B][max_steps] (drawn µ-law codes), "wav" fp32 [B][max_steps]
 * (mu_decode of the draws, imodel.py:181-182), "logits" [B][Q] (last step), "step" int64,
 * "rings" (lookback state, SAVE layout), "teacher" int32, "status" int32 (0; 5 when a persistent
 * hand-off timed out). */
int lbwn_gen_tensor(const lbwn_gen_plan* plan, const char* name, size_t* offset, size_t* bytes);
/* Reset the state (zero lookback rings = imodel's zero-initialised buffers, step 0 input =
 * zero vector), load the teacher codes (device int32, may be NULL) and GC ids (device
 * int32 [B], GC archs; imodel.py:53-56).  pre_bias=1 adds PRE_BIAS to the input embedding
 * (tmodel-consistent); 0 reproduces imodel.py:75-77 literally.  Draws use
 * u = splitmix64(seed, stream, step) >> 40 / 2^24 and the inverse softmax CDF (the
 * reference's tf.multinomial, imodel.py:179, is TF-RNG and not reproducible). */
int lbwn_gen_start(lbwn_gen_plan* plan, const lbwn_params* params, void* workspace, const int* gc_ids,
                   const int* teacher, int64_t n_teacher, uint64_t seed, int pre_bias, void* stream);
/* Generate n_steps more samples for every stream (the tf.while_loop body, imodel.py:214-272).
 * Device-resident step counter: the launches are graph-capturable and replayable.  Persistent
 * plans (lbwn_gen_is_persistent) run the whole call as ONE launch whose blocks must all be
 * resident: nothing else may occupy the device's CUs meanwhile. */
int lbwn_gen_run(lbwn_gen_plan* plan, const lbwn_params* params, void* workspace, int n_steps, void* stream);
/* 1 when the plan runs the persistent one-launch form (groups of <= 16 streams, each with its
 * own 32 head blocks, while every block fits on the device: B <= 80 on 256 CUs; layer/head sizes fit;
 * LBWN_GEN_PERSIST=0 at plan creation selects the per-step launches), else 0. */
int lbwn_gen_is_persistent(const lbwn_gen_plan* plan);

/* ---- fine-grained kernels (parity tests, custom drivers) ------------------------------ */
/* ops.mu_encode_np (ops.py:23-28, tf32=0, float64 math) / ops.mu_encode (ops.py:4-9, tf32=1) */
int lbwn_mulaw_encode(const float* x, int* q, int64_t n, int n_quanta, int tf32, void* stream);
/* ops.mu_decode (ops.py:12-20) */
int lbwn_mulaw_decode(const int* q, float* x, int64_t n, int n_quanta, void* stream);

/* GEMM arithmetic for every lbwn 1x1 product (process-wide; not a reference interface).
 * mode 1 (default): f32 operands split exactly into three bf16 terms, six cross products on
 * the bf16 matrix cores, f32 accumulation (f32-class error, tests/test_gpu_parity.py
 * ::test_gemm_split_accuracy).  mode 0: v_mfma_f32_32x32x2_f32.  Env LBWN_GEMM=f32 sets 0. */
int lbwn_gemm_set_mode(int mode);
int lbwn_gemm_get_mode(void);

/* ops.conv1x1 and every 1x1 product (ops.py:41-55): C[M][N] = epi(A·B).
 * a_kcontig: A stored A[m*lda+k] (else A[k*lda+m]); b_kcontig: B stored B[n*ldb+k]
 * (else B[k*ldb+n]).  Epilogue: +bias[n], relu, zero where mask[m*ldm+n] <= 0, += C.
 * relu_a applies relu to A on load.  split_k > 1 needs slab_ws of split_k·M·N floats. */
int lbwn_gemm_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb, int b_kcontig,
                  float* C, int64_t ldc, int M, int N, int K, const float* bias, int relu_a, int relu_out,
                  const float* mask, int64_t ldm, int accumulate, int split_k, float* slab_ws, void* stream);

/* The same product with B given ALSO as pre-split bf16 planes b3 (lbwn_split_planes of B with
 * rows = N: trans = 0 for B[n*ldb+k], 1 for B[k*ldb+n]), the form the training step uses for its
 * weight operands; no split-K.  B stays required for the f32 mode (mode 0 ignores b3).
 * b3 must be 16-byte aligned (else EINVAL) and hold lbwn_split_planes_elems_abi(N, K) elements. */
int lbwn_gemm_f32_presplit(const float* A, int64_t lda, int a_kcontig, const uint16_t* b3, int N, const float* B,
                           int64_t ldb, int b_kcontig, float* C, int64_t ldc, int M, int K, const float* bias,
                           int relu_a, int relu_out, const float* mask, int64_t ldm, int accumulate, void* stream);
/* Exact three-term bf16 split of a weight, out[r][K/32][3][32] (K rounded up to 32, zero-filled):
 * W[r*ldw+k] (trans = 0) or W[k*ldw+r] (trans = 1), r < rows. */
int64_t lbwn_split_planes_elems_abi(int rows, int K);
int lbwn_split_planes(const float* W, int64_t ldw, int rows, int K, int trans, uint16_t* out, void* stream);

/* One residual layer forward (tmodel.py:117-184): x_in is the [B][H+T][n_res] halo
 * buffer whose rows [H-d, H) hold SAVE; writes z [M][*] (row stride ldz) and, if x_out,
 * x_out body rows (x + z·RES + b). gc_tab [n_cat+1][2·n_dil] / ids, cond [M][2·n_dil]
 * (row stride ldcond) are optional conditioning adds.  wpack_ws: 16-B aligned scratch of
 * lbwn_layer_image_floats_abi() floats for the packed weight image. */
int lbwn_layer_image_floats_abi(void);
int lbwn_layer_forward(const float* x_in, float* x_out, float* z, int64_t ldz, const float* w_sig,
                       const float* w_gate, const float* b_sig, const float* b_gate, const float* w_res,
                       const float* b_res, const float* gc_tab, const int* ids, const float* cond,
                       int64_t ldcond, int B, int T, int H, int dilation, int n_res, int n_dil, float* wpack_ws,
                       void* stream);

/* One residual layer backward: TF's autodiff of tmodel.py:117-184 for one layer (the SURVEY
 * §8b lbwn_dilconv_gate_bwd).  Inputs as lbwn_layer_forward plus dz = dL/dz from the skip path
 * ([M] rows, stride lddz) and dx_out = dL/dx_out of the layer's output x_{l+1} ([M][n_res], NULL
 * for the last layer).  Recomputes the gate from x_in.  Writes dx_in = dL/d(x_in) over the whole
 * [B][H+T][n_res] halo buffer (rows [H-d, H) are the SAVE rows' share; earlier rows 0), the
 * weight and bias gradients in the reference layouts (overwritten), dcond = dL/d(cond) ([M] rows
 * of 2·n_dil, stride lddcond) when cond is given, and adds into gc_dtab [ncat+1][2·n_dil] (per
 * voice id) when given.  ws: 16-B aligned scratch of lbwn_layer_backward_ws_floats() floats. */
int64_t lbwn_layer_backward_ws_floats(int B, int T, int n_res);
int lbwn_layer_backward(const float* x_in, const float* dz, int64_t lddz, const float* dx_out, const float* w_sig,
                        const float* w_gate, const float* b_sig, const float* b_gate, const float* w_res,
                        const float* b_res, const float* gc_tab, const int* ids, const float* cond, int64_t ldcond,
                        float* dx_in, float* dw_sig, float* dw_gate, float* db_sig, float* db_gate, float* dw_res,
                        float* db_res, float* dcond, int64_t lddcond, float* gc_dtab, int B, int T, int H, int dilation,
                        int n_res, int n_dil, float* ws, void* stream);

/* D-separation prepend/save for all layers at once (tmodel.py:122-127, :165). */
int lbwn_dsep_prepend(float* x_all, int64_t x_layer_stride, const float* save, int n_layers, int n_block_layers,
                      int B, int T, int H, int n_res, void* stream);
int lbwn_dsep_save(const float* x_all, int64_t x_layer_stride, float* save, int n_layers, int n_block_layers,
                   int B, int T, int H, int n_res, void* stream);

/* softmax_cross_entropy_with_logits_v2 on logits[:, :-1] vs one-hot(wav_q[:, 1:]) with
 * mask ids[:, 1:] != 0 (tmodel.py:228-249).  Overwrites logits with the unnormalised
 * gradient (softmax - onehot)·mask when write_grad; stats as lbwn_train_forward.
 * partial_ws: 3·2048 floats. */
int lbwn_head_xent(float* logits, const int* wav_q, const int* ids, int B, int T, int Q, int write_grad,
                   float* stats, float* partial_ws, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LBWN_H */
