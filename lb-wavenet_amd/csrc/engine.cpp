// lbwn plan: the WaveNetTrain training graph (tmodel.py:292-340) as a fixed sequence of
// HIP launches over one caller-owned workspace.  Replaces TF's graph executor for this
// path: the 50-layer loop that TF unrolls at graph-build time (tmodel.py:313-325) is a
// native loop here, every buffer is carved once at plan creation, and nothing allocates
// or synchronises inside forward/backward (so a caller may capture them in a hipGraph).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <new>

#include "../../include/lbwn.h"
#include "common.h"
#include "kernels.h"

struct lbwn_plan {
  lbwn_arch a;
  int B, T, L, nbl, H, Cr, Cd, Cs, Cp, Q;
  long M;
  // workspace carving (byte offsets)
  size_t oX, oZ, oS, oR2, oLOG, oGA[2], oGC0[2], oDX0, oSLAB[2], oSPLIT, oCOLS, oHEADP, oBSUM, oWPK;
  size_t total;
  long x_layer_stride;  // floats
  int split_post2, split_post1, split_skip, split_pre;
  long split_floats;
  // one-shot event probe
  char probe[32];
  hipEvent_t probe_start, probe_stop;
};

namespace {
struct Probe {
  lbwn_plan* p;
  hipStream_t st;
  bool on;
  // name: launch kind; l: layer index (-1 = not a layer launch); first/last: span of a kind
  Probe(lbwn_plan* p_, hipStream_t s, const char* name, int l = -1, bool first = true) : p(p_), st(s), on(false) {
    if (!p->probe[0]) return;
    char full[40];
    snprintf(full, sizeof(full), "%s@%d", name, l);
    if (!strcmp(p->probe, full) || (!strcmp(p->probe, name) && first)) {
      (void)hipEventRecord(p->probe_start, st);
    }
  }
  static void end(lbwn_plan* p, hipStream_t st, const char* name, int l = -1, bool last = true) {
    if (!p->probe[0]) return;
    char full[40];
    snprintf(full, sizeof(full), "%s@%d", name, l);
    if (!strcmp(p->probe, full) || (!strcmp(p->probe, name) && last)) {
      (void)hipEventRecord(p->probe_stop, st);
      p->probe[0] = 0;
    }
  }
};
}  // namespace

int lbwn_plan_probe(lbwn_plan* p, const char* name, void* ev_start, void* ev_stop) {
  LBWN_REQUIRE(p && name && ev_start && ev_stop, "plan_probe: null argument");
  LBWN_REQUIRE(strlen(name) < sizeof(p->probe), "plan_probe: name too long");
  strcpy(p->probe, name);
  p->probe_start = (hipEvent_t)ev_start;
  p->probe_stop = (hipEvent_t)ev_stop;
  return 0;
}

namespace {

size_t carve(size_t& cur, size_t bytes) {
  size_t o = cur;
  cur += (bytes + 255) / 256 * 256;
  return o;
}

// Split-K for the weight-gradient GEMMs (K = B·T positions).  One 4-wave block per CU
// leaves the MFMA pipe latency-exposed, so aim for ~4 resident blocks per CU (1024 blocks)
// with the slab traffic capped at 64 MB.
int pick_split(int M, int N, long K) {
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  const long slab_cap = std::max<long>(1, (64L << 20) / (4L * M * N));
  const long s = std::max<long>(1, std::min<long>({1024 / tiles, K / 512, slab_cap}));
  return (int)s;
}

template <typename T>
T* at(void* ws, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}

}  // namespace

int lbwn_recep_field_sz(const lbwn_arch* a) {
  int s = 0;
  for (int l = 0; l < a->n_block_layers; ++l) s += 1 << l;
  return a->n_blocks * s;
}

int lbwn_plan_create(const lbwn_arch* a, int B, int T, lbwn_plan** out) {
  LBWN_REQUIRE(a && out, "plan_create: null argument");
  LBWN_REQUIRE(a->n_blocks >= 1 && a->n_block_layers >= 1 && a->n_block_layers <= 16, "plan: bad depth");
  LBWN_REQUIRE(a->n_res >= 1 && a->n_res <= 32 && a->n_dil >= 1 && a->n_dil <= 32,
               "plan: n_res/n_dil must be in [1, 32] (got %d/%d)", a->n_res, a->n_dil);
  LBWN_REQUIRE(a->n_skip % 4 == 0 && a->n_post % 4 == 0 && a->n_quant % 4 == 0,
               "plan: n_skip/n_post/n_quant must be multiples of 4");
  LBWN_REQUIRE(B >= 1 && T >= 2, "plan: batch_sz >= 1 and slice_sz >= 2 required");
  LBWN_REQUIRE(a->n_gc_embed == 0 && a->n_lc_out == 0, "plan: GC/LC conditioning not yet supported by this build");
  lbwn_plan* p = new (std::nothrow) lbwn_plan();
  LBWN_REQUIRE(p, "plan: out of host memory");
  p->a = *a;
  p->B = B;
  p->T = T;
  p->nbl = a->n_block_layers;
  p->L = a->n_blocks * a->n_block_layers;
  p->H = 1 << (a->n_block_layers - 1);
  p->Cr = a->n_res;
  p->Cd = a->n_dil;
  p->Cs = a->n_skip;
  p->Cp = a->n_post;
  p->Q = a->n_quant;
  p->M = (long)B * T;
  const long M = p->M;
  const int L = p->L;
  p->x_layer_stride = (long)B * (p->H + T) * p->Cr;
  // keep every x row 16-B aligned for the vector path
  p->x_layer_stride = (p->x_layer_stride + 3) / 4 * 4;
  const long ldz = (long)L * p->Cd;
  p->split_post2 = pick_split(p->Cp, p->Q, M);
  p->split_post1 = pick_split(p->Cs, p->Cp, M);
  p->split_skip = pick_split(L * p->Cd, p->Cs, M);
  p->split_pre = pick_split(p->Q, p->Cr, M);
  p->split_floats = std::max({(long)p->split_post2 * p->Cp * p->Q, (long)p->split_post1 * p->Cs * p->Cp,
                              (long)p->split_skip * ldz * p->Cs, (long)p->split_pre * p->Q * p->Cr});
  const int nblk = lbwn_layer_bwd_grid(B, T);
  size_t cur = 0;
  p->oX = carve(cur, sizeof(float) * (size_t)p->x_layer_stride * L);
  p->oZ = carve(cur, sizeof(float) * (size_t)M * ldz);
  p->oS = carve(cur, sizeof(float) * (size_t)M * p->Cs);
  p->oR2 = carve(cur, sizeof(float) * (size_t)M * p->Cp);
  p->oLOG = carve(cur, sizeof(float) * (size_t)M * p->Q);
  for (int i = 0; i < 2; ++i) {
    p->oGA[i] = carve(cur, sizeof(float) * (size_t)M * p->Cr);
    p->oGC0[i] = carve(cur, sizeof(float) * (size_t)M * p->Cr);
    p->oSLAB[i] = carve(cur, sizeof(float) * (size_t)nblk * lbwn_layer_slab_stride());
  }
  p->oDX0 = carve(cur, sizeof(float) * (size_t)M * p->Cr);
  p->oSPLIT = carve(cur, sizeof(float) * (size_t)p->split_floats);
  p->oCOLS = carve(cur, sizeof(float) * (size_t)lbwn_colsum_ws_floats((int)M, std::max({p->Cs, p->Cp, p->Q, p->Cr})));
  p->oHEADP = carve(cur, sizeof(float) * 3 * 2048);
  p->oBSUM = carve(cur, sizeof(float) * (size_t)p->Cs);
  p->oWPK = carve(cur, sizeof(float) * (size_t)L * lbwn_layer_image_floats());
  p->total = cur;
  *out = p;
  return 0;
}

void lbwn_plan_destroy(lbwn_plan* p) { delete p; }

int lbwn_plan_tensor(const lbwn_plan* p, const char* name, size_t* off, size_t* bytes) {
  LBWN_REQUIRE(p && name && off && bytes, "plan_tensor: null argument");
  const size_t M = (size_t)p->M, f = sizeof(float);
  if (!strcmp(name, "x")) { *off = p->oX; *bytes = f * (size_t)p->x_layer_stride * p->L; }
  else if (!strcmp(name, "z")) { *off = p->oZ; *bytes = f * M * p->L * p->Cd; }
  else if (!strcmp(name, "s")) { *off = p->oS; *bytes = f * M * p->Cs; }
  else if (!strcmp(name, "r2")) { *off = p->oR2; *bytes = f * M * p->Cp; }
  else if (!strcmp(name, "logits")) { *off = p->oLOG; *bytes = f * M * p->Q; }
  else LBWN_REQUIRE(false, "plan_tensor: unknown tensor '%s'", name);
  return 0;
}
size_t lbwn_plan_workspace_bytes(const lbwn_plan* p) { return p ? p->total : 0; }

static lbwn_gemm_args gemm0() {
  lbwn_gemm_args g;
  memset(&g, 0, sizeof(g));
  return g;
}

int lbwn_train_forward(lbwn_plan* p, const lbwn_params* P, void* ws, const int* wav_q, const int* ids,
                       const float* mel, float* save, float* stats, void* stream) {
  LBWN_REQUIRE(p && P && ws && wav_q && ids && save && stats, "train_forward: null argument");
  (void)mel;
  hipStream_t st = (hipStream_t)stream;
  const int L = p->L, B = p->B, T = p->T, H = p->H, Cr = p->Cr, Cd = p->Cd;
  const long M = p->M, ldz = (long)L * Cd;
  float* X = at<float>(ws, p->oX);
  float* Z = at<float>(ws, p->oZ);
  float* S = at<float>(ws, p->oS);
  float* R2 = at<float>(ws, p->oR2);
  float* LOG = at<float>(ws, p->oLOG);
  float* bsum = at<float>(ws, p->oBSUM);
  int e;
  // per-layer weights -> padded LDS images (once per step; reused by the backward)
  float* WPK = at<float>(ws, p->oWPK);
  if ((e = lbwn_pack_layers_launch(P->sig, P->gate, P->sig_b, P->gate_b, P->res, P->res_b, WPK, L, Cr, Cd, st)))
    return e;
  // one-hot·PRE + PRE_BIAS == row gather (tmodel.py:53-66, :86-102)
  if ((e = lbwn_embed_launch(wav_q, P->pre, P->pre_b, X, B, T, H, Cr, p->Q, st))) return e;
  // D-separation prepend for every layer (tmodel.py:122-127)
  if ((e = lbwn_dsep_prepend_launch(X, p->x_layer_stride, save, L, p->nbl, B, T, H, Cr, st))) return e;
  for (int l = 0; l < L; ++l) {
    lbwn_layer_args a;
    memset(&a, 0, sizeof(a));
    a.x_in = X + l * p->x_layer_stride;
    a.x_out = (l + 1 < L) ? X + (l + 1) * p->x_layer_stride : nullptr;
    a.z = Z + (long)l * Cd;
    a.ldz = ldz;
    a.w_sig = P->sig + (long)l * 2 * Cr * Cd;
    a.w_gate = P->gate + (long)l * 2 * Cr * Cd;
    a.b_sig = P->sig_b ? P->sig_b + (long)l * Cd : nullptr;
    a.b_gate = P->gate_b ? P->gate_b + (long)l * Cd : nullptr;
    a.w_res = P->res + (long)l * Cd * Cr;
    a.b_res = P->res_b ? P->res_b + (long)l * Cr : nullptr;
    a.wpack = WPK + (long)l * lbwn_layer_image_floats();
    a.ids = ids;
    a.B = B;
    a.T = T;
    a.H = H;
    a.d = 1 << (l % p->nbl);
    a.Cr = Cr;
    a.Cd = Cd;
    Probe(p, st, "layer_fwd", l, l == 0);
    if ((e = lbwn_layer_fwd_launch(a, st))) return e;
    Probe::end(p, st, "layer_fwd", l, l == L - 1);
  }
  // SAVE_l <- last d rows of [SAVE ++ x_l]  (tmodel.py:165)
  if ((e = lbwn_dsep_save_launch(X, p->x_layer_stride, save, L, p->nbl, B, T, H, Cr, st))) return e;
  // S = Σ_l (z_l·SKIP_l + b) as ONE GEMM over Zcat (tmodel.py:171-184, :316-320)
  lbwn_gemm_args g = gemm0();
  if (P->skip_b) {
    if ((e = lbwn_sum_bias_launch(P->skip_b, L, p->Cs, bsum, st))) return e;
  }
  g.A = Z; g.lda = ldz; g.B = P->skip; g.ldb = p->Cs; g.C = S; g.ldc = p->Cs;
  g.M = (int)M; g.N = p->Cs; g.K = (int)ldz; g.bias = P->skip_b ? bsum : nullptr;
  Probe(p, st, "skip_fwd");
  if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
  Probe::end(p, st, "skip_fwd");
  // relu(relu(S)·POST1 + b1)  (tmodel.py:194-203)
  g = gemm0();
  g.A = S; g.lda = p->Cs; g.B = P->post1; g.ldb = p->Cp; g.C = R2; g.ldc = p->Cp;
  g.M = (int)M; g.N = p->Cp; g.K = p->Cs; g.bias = P->post1_b; g.relu_a = 1; g.relu_out = 1;
  Probe(p, st, "post1_fwd");
  if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
  Probe::end(p, st, "post1_fwd");
  // logits = R2·POST2 + b2  (tmodel.py:204-209)
  g = gemm0();
  g.A = R2; g.lda = p->Cp; g.B = P->post2; g.ldb = p->Q; g.C = LOG; g.ldc = p->Q;
  g.M = (int)M; g.N = p->Q; g.K = p->Cp; g.bias = P->post2_b;
  Probe(p, st, "post2_fwd");
  if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
  Probe::end(p, st, "post2_fwd");
  // masked softmax-xent (+ unnormalised dlogits in place)  (tmodel.py:228-249)
  lbwn_head_args h;
  h.logits = LOG; h.q = wav_q; h.ids = ids; h.B = B; h.T = T; h.Q = p->Q;
  h.partial = at<float>(ws, p->oHEADP); h.write_grad = 1;
  int nb = 0;
  Probe(p, st, "head");
  if ((e = lbwn_head_launch(h, &nb, st))) return e;
  Probe::end(p, st, "head");
  return lbwn_stats_reduce_launch(h.partial, nb, stats, st);
}

int lbwn_train_backward(lbwn_plan* p, const lbwn_params* P, const lbwn_params* G, void* ws, const int* wav_q,
                        const int* ids, const float* mel, void* stream) {
  LBWN_REQUIRE(p && P && G && ws && wav_q && ids, "train_backward: null argument");
  (void)mel;
  hipStream_t st = (hipStream_t)stream;
  const int L = p->L, B = p->B, T = p->T, H = p->H, Cr = p->Cr, Cd = p->Cd, Cs = p->Cs, Cp = p->Cp, Q = p->Q;
  const long M = p->M, ldz = (long)L * Cd;
  float* X = at<float>(ws, p->oX);
  float* Z = at<float>(ws, p->oZ);
  float* S = at<float>(ws, p->oS);
  float* R2 = at<float>(ws, p->oR2);
  float* LOG = at<float>(ws, p->oLOG);
  float* SPL = at<float>(ws, p->oSPLIT);
  float* COLS = at<float>(ws, p->oCOLS);
  int e;
  lbwn_gemm_args g;
  // dPOST2 = R2ᵀ·dlogits, db2 = Σ dlogits
  g = gemm0();
  g.A = R2; g.lda = Cp; g.B = LOG; g.ldb = Q; g.C = G->post2; g.ldc = Q; g.M = Cp; g.N = Q; g.K = (int)M;
  Probe(p, st, "dpost2");
  if ((e = lbwn_gemm_launch(g, 0, 0, p->split_post2, SPL, st))) return e;
  Probe::end(p, st, "dpost2");
  if (G->post2_b && (e = lbwn_colsum_launch(LOG, Q, (int)M, Q, G->post2_b, 0, COLS, st))) return e;
  // dH1 = dlogits·POST2ᵀ ⊙ (R2 > 0)   (in place over R2)
  g = gemm0();
  g.A = LOG; g.lda = Q; g.B = P->post2; g.ldb = Q; g.C = R2; g.ldc = Cp; g.M = (int)M; g.N = Cp; g.K = Q;
  g.mask = R2; g.ldm = Cp;
  if ((e = lbwn_gemm_launch(g, 1, 1, 1, nullptr, st))) return e;
  // dPOST1 = relu(S)ᵀ·dH1, db1 = Σ dH1
  g = gemm0();
  g.A = S; g.lda = Cs; g.relu_a = 1; g.B = R2; g.ldb = Cp; g.C = G->post1; g.ldc = Cp; g.M = Cs; g.N = Cp;
  g.K = (int)M;
  Probe(p, st, "dpost1");
  if ((e = lbwn_gemm_launch(g, 0, 0, p->split_post1, SPL, st))) return e;
  Probe::end(p, st, "dpost1");
  if (G->post1_b && (e = lbwn_colsum_launch(R2, Cp, (int)M, Cp, G->post1_b, 0, COLS, st))) return e;
  // dS = dH1·POST1ᵀ ⊙ (S > 0)   (in place over S)
  g = gemm0();
  g.A = R2; g.lda = Cp; g.B = P->post1; g.ldb = Cp; g.C = S; g.ldc = Cs; g.M = (int)M; g.N = Cs; g.K = Cp;
  g.mask = S; g.ldm = Cs;
  if ((e = lbwn_gemm_launch(g, 1, 1, 1, nullptr, st))) return e;
  // dSKIPcat = Zcatᵀ·dS; every layer's SKIP_BIAS gets the same Σ dS
  g = gemm0();
  g.A = Z; g.lda = ldz; g.B = S; g.ldb = Cs; g.C = G->skip; g.ldc = Cs; g.M = (int)ldz; g.N = Cs; g.K = (int)M;
  Probe(p, st, "dskip");
  if ((e = lbwn_gemm_launch(g, 0, 0, p->split_skip, SPL, st))) return e;
  Probe::end(p, st, "dskip");
  if (G->skip_b) {
    if ((e = lbwn_colsum_launch(S, Cs, (int)M, Cs, G->skip_b, 0, COLS, st))) return e;
    if ((e = lbwn_bcast_rows_launch(G->skip_b, L, Cs, st))) return e;
  }
  // dZ = dS·SKIPcatᵀ  (over Z: z is recomputed by the layer backward)
  g = gemm0();
  g.A = S; g.lda = Cs; g.B = P->skip; g.ldb = Cs; g.C = Z; g.ldc = ldz; g.M = (int)M; g.N = (int)ldz; g.K = Cs;
  Probe(p, st, "dz");
  if ((e = lbwn_gemm_launch(g, 1, 1, 1, nullptr, st))) return e;
  Probe::end(p, st, "dz");
  // residual stack in reverse; layer l reduces layer l+1's weight-grad partials on the fly
  const int nblk = lbwn_layer_bwd_grid(B, T);
  const float* WPK = at<float>(ws, p->oWPK);
  for (int l = L - 1; l >= 0; --l) {
    lbwn_layer_args a;
    memset(&a, 0, sizeof(a));
    a.x_in = X + l * p->x_layer_stride;
    a.w_sig = P->sig + (long)l * 2 * Cr * Cd;
    a.w_gate = P->gate + (long)l * 2 * Cr * Cd;
    a.b_sig = P->sig_b ? P->sig_b + (long)l * Cd : nullptr;
    a.b_gate = P->gate_b ? P->gate_b + (long)l * Cd : nullptr;
    a.w_res = P->res + (long)l * Cd * Cr;
    a.b_res = P->res_b ? P->res_b + (long)l * Cr : nullptr;
    a.wpack = WPK + (long)l * lbwn_layer_image_floats();
    a.ids = ids;
    a.B = B; a.T = T; a.H = H; a.d = 1 << (l % p->nbl); a.Cr = Cr; a.Cd = Cd;
    a.dz_skip = Z + (long)l * Cd;
    a.lddz = ldz;
    if (l + 1 < L) {
      a.g_a = at<float>(ws, p->oGA[(l + 1) & 1]);
      a.g_c0 = at<float>(ws, p->oGC0[(l + 1) & 1]);
      a.g_d = 1 << ((l + 1) % p->nbl);
      const int lp = l + 1;
      a.red_slab = at<float>(ws, p->oSLAB[lp & 1]);
      a.red_nparts = nblk;
      a.red_stride = lbwn_layer_slab_stride();
      a.red_dsig = G->sig + (long)lp * 2 * Cr * Cd;
      a.red_dgate = G->gate + (long)lp * 2 * Cr * Cd;
      a.red_dres = G->res + (long)lp * Cd * Cr;
      a.red_dbsig = G->sig_b ? G->sig_b + (long)lp * Cd : nullptr;
      a.red_dbgate = G->gate_b ? G->gate_b + (long)lp * Cd : nullptr;
      a.red_dbres = G->res_b ? G->res_b + (long)lp * Cr : nullptr;
    }
    a.out_a = at<float>(ws, p->oGA[l & 1]);
    a.out_c0 = at<float>(ws, p->oGC0[l & 1]);
    a.slab = at<float>(ws, p->oSLAB[l & 1]);
    a.slab_stride = lbwn_layer_slab_stride();
    Probe(p, st, "layer_bwd", l, l == L - 1);
    if ((e = lbwn_layer_bwd_launch(a, st))) return e;
    Probe::end(p, st, "layer_bwd", l, l == 0);
  }
  {  // layer 0's partials
    lbwn_layer_args a;
    memset(&a, 0, sizeof(a));
    a.Cr = Cr; a.Cd = Cd;
    a.red_slab = at<float>(ws, p->oSLAB[0]);
    a.red_nparts = nblk;
    a.red_stride = lbwn_layer_slab_stride();
    a.red_dsig = G->sig; a.red_dgate = G->gate; a.red_dres = G->res;
    a.red_dbsig = G->sig_b; a.red_dbgate = G->gate_b; a.red_dbres = G->res_b;
    if ((e = lbwn_layer_reduce_launch(a, st))) return e;
  }
  // dx_0 = (g + dcur) + shift(dprev); dPRE = onehot(q)ᵀ·dx_0, dPRE_BIAS = Σ dx_0
  float* DX0 = at<float>(ws, p->oDX0);
  if ((e = lbwn_shift_add_launch(DX0, at<float>(ws, p->oGA[0]), at<float>(ws, p->oGC0[0]), 1, B, T, Cr, st)))
    return e;
  g = gemm0();
  g.a_codes = wav_q; g.B = DX0; g.ldb = Cr; g.C = G->pre; g.ldc = Cr; g.M = Q; g.N = Cr; g.K = (int)M;
  g.lda = 4;  // unused (one-hot A)
  if (Cr % 4 == 0) {
    if ((e = lbwn_gemm_launch(g, 0, 0, p->split_pre, SPL, st))) return e;
  } else {
    LBWN_REQUIRE(false, "train_backward: n_res %% 4 != 0 not supported for the PRE gradient yet");
  }
  if (G->pre_b && (e = lbwn_colsum_launch(DX0, Cr, (int)M, Cr, G->pre_b, 0, COLS, st))) return e;
  return 0;
}
