// Internal launch interfaces shared by the kernel TUs and the engine (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct lbwn_gemm_args {
  const float* A; long lda;
  const float* B; long ldb;
  float* C; long ldc;
  int M, N, K;
  const float* bias;   // [N] nullable
  const float* mask;   // mask[m*ldm+n] > 0 keeps the value; nullable
  long ldm;
  int relu_a, relu_out, accumulate;
  const unsigned short* b3;  // nullable: B pre-split into bf16 planes [N][K/32][3][32] (lbwn_split_planes_launch)
  const int* a_codes;  // m-contiguous A only: A[k][m] = (a_codes[k] == m)  (one-hot, tmodel.py:64-65)
  // nullable, bf16-split form without split-K only: column partial sums of the final C values
  // (after bias/relu/mask), [ceil(M/256)][N] (one part per 256-row block tile), summed by
  // lbwn_colsum_final_launch: the bias gradient without a second pass over C
  float* colpart;
  long long* step_advance;   // nullable, bf16-split form only: block 0 adds 1 (the per-step generator's counter)
  // bf16-split form, no split-K / accumulate / mask: > 0 stores C in the backward chain's row-load
  // order instead of rows (ldc unused): 32-column block j at C + j·c_chain_ls, element (m, c) at
  // sg_off(m, c / 8, (c / 4) & 1) + c % 4 (layer.hip), so the chain's own-row loads are 1-KiB runs
  long c_chain_ls;
  int k_per_split;     // set by the launcher
  int* splits_deferred;   // host, nullable: split-K partials left unsummed in the slab workspace
                          // ([splits][M][N]); the launcher stores the split count here (1: C written)
  long split_stride;   // set by the launcher
  int xcd2d;           // gemm_x3q_kernel<10> (N % 160 == 0): the 2-D XCD blocking of its tiles (xcd2d_tile)
  // k-blocked operands (the backward chain's DV export, [K/32][Mp][32]): 0 = plain layout.
  // a_kstride: A k-contiguous with lda = 32, element (m, k) at A[m·32 + (k/32)·a_kstride + k%32]
  // (gemm_x3q_kernel only); b_gstride: B mn-contiguous with ldb = 32, element (k, n) at
  // B[k·32 + (n/32)·b_gstride + n%32] (the LDS-staged bf16-split kernel only); a_gstride: A
  // mn-contiguous with lda = 32, element (m, k) at A[k·32 + (m/32)·a_gstride + m%32] (the AMN
  // form of gemm_x3q_kernel only: dLCcat as DVᵀ·lc)
  long a_kstride, b_gstride, a_gstride;
  // 1: every output row is computed by the same kernel and k order whatever M is (the tall
  // 256-row form below M = 8192 too), so a row's value depends only on its own A row: the
  // training forward's head GEMMs, so a slice processed in stages equals one long slice bit for
  // bit (README.md:6-21)
  int row_exact;
  // gemm_x3q_kernel<8> tile form (lbwn_gemm_x3q8_form) only: the relu / mask predicate of the C
  // values as one 64-bit word per lane ([tile][wave][lane]: bit 8·nb + e = element (e, nb) of the
  // lane's epilogue), so a later GEMM of the SAME shape and form masks by it (mbits) instead of
  // reading an f32 M×N mask: mbits_out (producer) sets bit = (final C > 0); mbits (consumer)
  // replaces mask.  lbwn_gemm_mbits_words(M, N) words each.
  unsigned long long* mbits_out;
  const unsigned long long* mbits;
};
// the tall pre-split product that runs gemm_x3q_kernel<8> (the form mbits / mbits_out need)
bool lbwn_gemm_x3q8_form(int M, int N, int K, int a_kcontig, int presplit, int row_exact, int colpart);
inline long lbwn_gemm_mbits_words(long M, long N) { return ((M + 255) / 256) * ((N + 127) / 128) * 8 * 64; }
int lbwn_gemm_launch(const lbwn_gemm_args& a, int a_kcontig, int b_kcontig, int split_k, float* slab_ws,
                     hipStream_t st);
inline int lbwn_colpart_parts(long M) { return (int)((M + 255) / 256); }
// Pre-split planes of a weight for lbwn_gemm_args::b3: rows = N of the product it feeds,
// W[r][k] (trans = 0) or W[k][r] (trans = 1), row stride ldw; up to 6 weights per launch.
// Element count of one output:
size_t lbwn_split_planes_elems(int rows, int K);
int lbwn_split_planes_launch(int njobs, const float* const* W, const long* ldw, const int* rows, const int* K,
                             const int* trans, unsigned short* const* out, hipStream_t st);
// 1: bf16-split (default), 0: f32 MFMA (gemm.hip)
int lbwn_gemm_mode(void);
int lbwn_gemm_set_mode_impl(int mode);
// same product with a 21 KB LDS footprint (BK = 8) so it can co-reside with a chain block
int lbwn_gemm_launch_lean(const lbwn_gemm_args& a, int a_kcontig, int b_kcontig, int split_k, float* slab_ws,
                          hipStream_t st);

// One residual layer (tmodel.py:117-184).  x buffers are [B][H+T][Cr]; rows [H-d, H) of
// x_in hold the D-separation state SAVE_l (prepended by lbwn_dsep_prepend).
struct lbwn_layer_args {
  const float* x_in;
  float* x_out;             // nullable (last layer's residual output is dead)
  float* z; long ldz;       // Zcat column block of this layer
  const float* w_sig; const float* w_gate;  // [2][Cr][Cd]
  const float* b_sig; const float* b_gate;  // [Cd] nullable
  const float* w_res; const float* b_res;   // [Cd][Cr], [Cr] nullable
  const float* wpack;       // packed LDS image of this layer (lbwn_pack_layers_launch)
  const float* gc_tab;      // rows [ncat+1] of (sig Cd | gate Cd), row stride gc_ld (0 = 2Cd); nullable
  long gc_ld;
  const int* ids;           // [B][T]
  const float* cond; long ldcond;  // [M][2*Cd] nullable (LC projection)
  int B, T, H, d, Cr, Cd;
  // ---- backward only ----
  const float* dz_skip; long lddz;   // [M] rows of dS·SKIP_lᵀ (column block of dZ)
  const float* g_a; const float* g_c0; int g_d;  // dx_{l+1}[t] = g_a[t] + g_c0[t+g_d]; nullable => 0
  float* out_a; float* out_c0;                    // [M][Cr]
  float* slab;              // per-block weight-grad partials [nblocks][slab_stride]
  int slab_stride;
  float* dv_out; long lddv; // [M][2Cd] nullable (needed for LC grads)
  float* gc_dtab;           // [ncat+1][2Cd] atomically accumulated (nullable)
};
// Sum a layer's per-block weight-grad partials into the reference-layout gradients.
struct lbwn_layer_red_args {
  const float* slab; int nparts; int stride;
  float* dsig; float* dgate; float* dres;      // [2][Cr][Cd], [2][Cr][Cd], [Cd][Cr]
  float* dbsig; float* dbgate; float* dbres;   // nullable
  int Cr, Cd;
};
constexpr int LBWN_LAYER_POS = 128;   // positions per layer-kernel block
int lbwn_layer_fwd_launch(const lbwn_layer_args& a, hipStream_t st);
int lbwn_layer_bwd_launch(const lbwn_layer_args& a, hipStream_t st);
int lbwn_layer_slab_stride();
// split weight images for the forward chain's bf16-split products (bf16 elements per layer)
int lbwn_layer_image_x3_elems();
// lbwn_pack_layers_x3_launch + lbwn_pack_layers_bx3_launch in one launch, plus (skip_b, bsum
// non-null) bsum[n] = Σ_l skip_b[l·Cs + n] (lbwn_sum_bias_launch)
// ... and (lcout non-null) the L split LC images of the in-chain LC term (lbwn_lc_image_x3_elems each)
// The training step's start-of-step work in one launch (layer.hip step_prologue_kernel): the
// arguments of lbwn_pack_layers_fb_x3_launch, lbwn_split_planes_launch (njobs 0..6),
// lbwn_embed_launch, lbwn_dsep_prepend_launch and lbwn_zero_launch (zero_bytes may be 0).
struct lbwn_prologue_args {
  const float *sig, *gate, *sig_b, *gate_b, *res, *res_b;
  unsigned short* fout;
  float* bout;
  int L, Cr, Cd;
  const float* skip_b;
  int Cs;
  float* bsum;
  const float *lc_sig, *lc_gate;
  int Lo;
  unsigned short* lcout;
  int lc16;
  int njobs;
  const float* W[6];
  long ldw[6];
  int rows[6], K[6], trans[6];
  unsigned short* out[6];
  const int* q;
  const float *pre, *pre_b;
  float* X;
  long xls;
  const float* save;
  int nbl, B, T, H, Q;
  void* zero;
  size_t zero_bytes;
};
int lbwn_step_prologue_launch(const lbwn_prologue_args& a, hipStream_t st);
int lbwn_pack_layers_fb_x3_launch(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                                  const float* res, const float* res_b, unsigned short* fout, float* bout, int L,
                                  int Cr, int Cd, const float* skip_b, int Cs, float* bsum, const float* lc_sig,
                                  const float* lc_gate, int Lo, unsigned short* lcout, hipStream_t st,
                                  int lc16 = 0);
int lbwn_lc_image_x3_elems();
int lbwn_lc_image16_elems();       // the 16-lane forward chain's LC image (lc16 = 1 above)
// forward chain form: 0 = 32-position waves (chain_fwd_kernel, 128-position tiles), 4 / 8 =
// 16-position waves (chain_fwd16_kernel) with 4 / 8 waves = 64- / 128-position tiles
int lbwn_chain_fwd_tile(int fwd_nw);
int lbwn_lc_in_chain_ok(int Lo);   // n_lc_out the forward chain's in-chain LC term supports
int lbwn_pack_layers_x3_launch(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                               const float* res, const float* res_b, unsigned short* out, int L, int Cr, int Cd,
                               hipStream_t st);
int lbwn_layer_image_floats();
int lbwn_layer_dx_combine_launch(const float* out_a, const float* out_c0, float* dx, int B, int T, int H, int d, int C,
                                 hipStream_t st);
// backward split images (WD bf16 + Rs f32) for the bf16-split backward chain, floats per layer
int lbwn_layer_image_bx3_floats();
int lbwn_pack_layers_bx3_launch(const float* sig, const float* gate, const float* res, float* out, int L, int Cr,
                                int Cd, hipStream_t st);
int lbwn_layer_nblocks(int B, int T);
int lbwn_layer_bwd_grid(int B, int T);   // = number of slab partials per layer
int lbwn_pack_layers_launch(const float* sig, const float* gate, const float* sig_b, const float* gate_b,
                            const float* res, const float* res_b, float* out, int L, int Cr, int Cd, hipStream_t st);
int lbwn_layer_reduce_launch(const lbwn_layer_red_args& r, hipStream_t st);

// Persistent layer chain (all L layers in one launch, tile hand-offs through flags).
struct lbwn_chain_args {
  float* X; long xls;          // x_l buffers of all layers, layer stride in floats
  float* Z; long ldz;
  const float* wpack;
  const unsigned short* wpack_x3;   // forward: split images (bf16-split conv/residual) or null
  const float* gc_tab; long gc_ld; const int* ids;   // GC table [ncat+1][L·2Cd] or null
  const float* cond; long ldcond;                     // LC term [M][L·2Cd] or null
  float* dv_out; long lddv; float* gc_dtab;           // backward: LC dv export, GC grad table
  unsigned* flags;             // [B·ceil(T/128)] (zeroed by the launcher unless flags_zeroed)
  int flags_zeroed;            // the caller zeroed flags on this stream (no memset here)
  unsigned* status;            // sticky error word (spin timeout)
  int B, T, H, L, nbl, Cr, Cd;
  int grid;                    // ≤ blocks resident at once (rounds of tiles)
  // backward only
  const float* DZ;             // dZ (row stride ldz), or in chain order (dzls > 0, bf16-split chain)
  long dzls = 0;               // chain order: layer stride of DZ (lbwn_gemm_args::c_chain_ls)
  float* slab;                 // [L][ntiles][slab_stride]
  float* ocg; long ocls;       // out_c0 hand-off rows per layer [L][B·T][32]
  float* dx0_a; float* dx0_c;  // layer 0's dx parts [B·T][32]
  long long* trace = nullptr;  // debug: cycle stamps of block trace_blk, [L][16] (LBWN_CHAIN_TRACE)
  int trace_blk = 0;
  // bf16-split backward (chain_bwd_x3_kernel): σ(v_gate) rows [L][M][32] written by the X3
  // forward chain (layer stride sgls floats), and the backward images (lbwn_pack_layers_bx3)
  float* SG = nullptr; long sgls = 0;
  const float* bimg = nullptr;
  int* tile_gid = nullptr;     // x3 backward + GC: [ntiles] uniform voice id per tile or -1
  float* gx = nullptr; long gxls = 0;   // chain_bwd16_kernel export form: G rows [L][Mp][32] (+ dv_out, dvks)
  // forward, bf16-split form: in-chain LC term (instead of cond): LC input [M][Lo], split images
  const float* lcact = nullptr; const unsigned short* lcimg = nullptr; int Lo = 0;
  int fwd_nw = 0;              // forward form (lbwn_chain_fwd_tile); lcimg in the matching layout
  int bwd_nw = 0;              // backward form: 0 = chain_bwd_x3_kernel (128), 4 / 8 = chain_bwd16_kernel
  int xcd = 0;                 // XCD-grouped tile walk (layer.hip chain_first)
  long dvks = 0;               // x3 backward forms: dv_out k-blocked ([L·2][Mp][32], chunk stride dvks)
};
int lbwn_chain_fwd_launch(const lbwn_chain_args& c, hipStream_t st);
int lbwn_chain_bwd_launch(const lbwn_chain_args& c, hipStream_t st);
int lbwn_layer_reduce_all_launch(const lbwn_layer_red_args& r, int L, long slab_layer, hipStream_t st);
// residual-stack weight-gradient partials from the backward chain's exports (layer_wgrad_kernel):
// slab [L][nchunk][stride] for lbwn_layer_reduce_all_launch (nparts = nchunk); GC (gcs non-null):
// tile ids + per-tile dv column sums [L][ntiles][64] for lbwn_gc_tile_sum_rows_launch
struct lbwn_wgrad_args {
  const float* X; long xls; const float* Z; long lddz;
  const float* DV; long dvks; const float* GX; long gxls;
  float* slab; long stride;
  const int* ids; int* tile_gid; float* gcs; float* gtab; long gc_ld;
  int B, T, H, L, nbl, tpc;
};
int lbwn_layer_wgrad_tiles_per_chunk(int ntiles, int L, int ncu);
int lbwn_layer_wgrad_launch(const lbwn_wgrad_args& g, hipStream_t st);
int lbwn_gc_tile_sum_rows_launch(const float* gcs, int L, int ntiles, const int* tile_gid, float* gtab, long ld,
                                 int ncat1, hipStream_t st);
int lbwn_chain_fwd_lds_bytes();

// D-separation state transfer for ALL layers at once.
int lbwn_dsep_prepend_launch(float* xall, long xlayer_stride, const float* save, int L, int nbl,
                             int B, int T, int H, int Cr, hipStream_t st);
int lbwn_dsep_save_launch(const float* xall, long xlayer_stride, float* save, int L, int nbl, int B,
                          int T, int H, int Cr, hipStream_t st);

int lbwn_embed_launch(const int* q, const float* pre, const float* pre_b, float* x0, int B, int T, int H,
                      int Cr, int Q, hipStream_t st);
int lbwn_embed_bwd_launch(const int* q, const float* ga, const float* gc0, int gd, float* dpre,
                          float* dpre_b, float* ws, int B, int T, int Cr, int Q, hipStream_t st);

struct lbwn_head_args {
  float* logits;            // [M][Q] in: logits, out: dlogits (unnormalised: (softmax-onehot)·mask)
  const int* q;             // [B][T] targets (mu-law codes)
  const int* ids;           // [B][T]
  int B, T, Q;
  float* partial;           // [nblocks][3] (sum_xent, n_valid, sum |argmax diff|)
  int write_grad;
  float* colpart;           // nullable: [nblocks][Q] column sums of the dlogits written (Q <= 512)
};
int lbwn_head_nblocks(long M, bool colpart);
int lbwn_head_launch(const lbwn_head_args& a, int* nblocks_out, hipStream_t st);
int lbwn_stats_reduce_launch(const float* partial, int nparts, float* stats, hipStream_t st);

// several column sums in one launch pair; ws holds Σ_j lbwn_colsum_ws_floats(M, N[j]) floats
int lbwn_colsum_multi_launch(int njobs, const float* const* X, const long* ldx, const int* N, float* const* out,
                             const int* accumulate, int M, float* ws, hipStream_t st);
int lbwn_colsum_launch(const float* X, long ldx, int M, int N, float* out, int accumulate, float* ws,
                       hipStream_t st);
int lbwn_colsum_ws_floats(int M, int N);
// the two passes apart: the first pass alone (*nparts = its partial row count; ws holds that ×
// N floats), and the second over any partials (first-pass ones or a GEMM epilogue's colpart)
int lbwn_colsum_partial_launch(const float* X, long ldx, int M, int N, float* ws, int* nparts, hipStream_t st);
int lbwn_colsum_final_launch(int njobs, float* const* parts, const int* N, float* const* out, const int* accumulate,
                             const int* nparts, hipStream_t st,
                             const int* reps = nullptr);
int lbwn_sum_bias_launch(const float* b, int L, int N, float* out, hipStream_t st);
int lbwn_fill_launch(float* p, float v, long n, hipStream_t st);

int lbwn_adam_launch2(float* params, const float* grads, float* m, float* v, long n_weights, long n_total,
                      float lr, float b1, float b2, float eps, float l2, const float* stats,
                      const long long* counters, const unsigned* status, hipStream_t st);
int lbwn_counters_launch(long long* counters, const float* stats, int adam_applied, const unsigned* status,
                         hipStream_t st);
// dPRE = onehot(q)ᵀ·dx0 as an LDS-histogram scatter + fixed-order reduction; dPRE_B = Σ dx0 (nullable);
// dx0[m] = g[m] + (t+gd < T ? dprev[m+gd] : 0) formed on the fly
int lbwn_pre_grad_ws_floats(int Q, int Cr);
int lbwn_pre_grad_launch(const int* q, const float* g, const float* dprev, int gd, int B, int T, int Cr, int Q,
                         float* dpre, float* dpre_b, float* ws, hipStream_t st);
int lbwn_shift_add_launch(float* out, const float* a, const float* c0, int gd, int B, int T, int C,
                          hipStream_t st);

int lbwn_mulaw_encode_launch(const float* x, int* q, long n, int n_quanta, int tf32, hipStream_t st);
int lbwn_mulaw_decode_launch(const int* q, float* x, long n, int n_quanta, hipStream_t st);
int lbwn_bcast_rows_launch(float* dst, int L, int N, hipStream_t st);
int lbwn_zero_launch(void* p, size_t n_bytes, hipStream_t st);
// GC table gradient of the uniform-id tiles from the backward chain's slab bias partials
int lbwn_gc_tile_sum_launch(const float* slab, int L, int ntiles, const int* tile_gid, float* gtab, long ld,
                            int ncat1, hipStream_t st);

// Conditioning (cond.hip)
int lbwn_gc_table_launch(const float* emb, const float* wsig, const float* wgate, float* out, int L, int ncat1,
                         int Ge, int Cd, hipStream_t st);
int lbwn_gc_grad_launch(const float* emb, const float* wsig, const float* wgate, const float* gcd, float* part,
                        float* demb, float* dsig, float* dgate, int L, int ncat1, int Ge, int Cd, hipStream_t st);
int lbwn_gc_part_floats(int L, int Ge, int Cd);
int lbwn_lc_pack_launch(float* cat, float* wsig, float* wgate, int L, int Clc, int Cd, int pack, hipStream_t st);
// LC upsample (tmodel.py:68-83) fused over its stages, one block per mel frame (cond.hip)
int lbwn_lc_up_fused_ok(int nup, const int* s, int Li, int Lo);
int lbwn_lc_up_part_floats(int nup, const int* s, int Li, int Lo, int frames);
int lbwn_lc_up_fwd_launch(int nup, const int* s, int Li, int Lo, int frames, const float* mel, const float* const* F,
                          float* const* act, hipStream_t st);
// the per-frame pass on st; the frame-partial sum on st_sum (after ev, recorded on st, when they differ)
int lbwn_lc_up_bwd_launch(int nup, const int* s, int Li, int Lo, int frames, const float* mel, const float* const* F,
                          float* const* act, const float* dlc, float* dpart, float* const* dF, hipStream_t st,
                          hipStream_t st_sum = nullptr, hipEvent_t ev = nullptr, int dlc_parts = 1,
                          long dlc_stride = 0);
