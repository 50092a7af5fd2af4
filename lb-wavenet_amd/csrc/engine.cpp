// lbwn plan: the WaveNetTrain training graph (tmodel.py:292-340) as a fixed sequence of
// HIP launches over one caller-owned workspace.  Replaces TF's graph executor for this
// path: the 50-layer loop that TF unrolls at graph-build time (tmodel.py:313-325) is a
// native loop here, every buffer is carved once at plan creation, and nothing allocates
// or synchronises inside forward/backward (so a caller may capture them in a hipGraph).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>

#include "../../include/lbwn.h"
#include "common.h"
#include "kernels.h"

struct lbwn_plan {
  int chain_xcd = 0;       // chain_first's XCD-grouped walk
  int dz_xcd2d = 1;        // dZ's tiles blocked 2-D over the XCDs (gemm.hip xcd2d_tile)
  int fwd_mode = -1;       // GEMM arithmetic (lbwn_gemm_mode) the last forward ran; the backward follows it
  int ncu = 0;             // compute units (ensure_device)
  // (S > 0) and (R2 > 0) as GEMM mask bits (lbwn_gemm_args::mbits): written by the skip / post1
  // epilogues, read by dS / dH1 instead of the f32 S / R2; set by the forward when both ends take
  // the gemm_x3q_kernel<8> form
  size_t oMBS = 0, oMBR = 0;
  bool mb_s = false, mb_r = false;
  bool mbits_ok = true;
  bool dv_blk = false;     // the last backward exported DV k-blocked ([2L][m32(M)][32])
  int head_colparts = 0;   // post2-bias column partial rows the last forward's head wrote (0: none)
  lbwn_arch a;
  int B, T, L, nbl, H, Cr, Cd, Cs, Cp, Q;
  int Ge, ncat1, Li, Lo, nup, hop, up[8];   // conditioning (Ge = 0: no GC, Lo = 0: no LC)
  long M;
  // workspace carving (byte offsets)
  size_t oCPART = 0, nflag_bytes = 0;
  bool bwd_flags_fresh = false;   // the step-start memset zeroed the backward flags, not yet used
  size_t oX, oZ, oS, oR2, oLOG, oDH, oDS, oDZ, oGA[2], oGC0[2], oSLAB, oSPLIT, oSPLIT2, oCOLS,
      oHEADP, oBSUM, oWPK, oWPKX, oFLAGS, oSTATUS, oOCG, oCTRACE;
  // bf16-split backward chain: σ(v_gate) rows from the forward chain [L][M][32], backward images
  size_t oSG = 0, oWPKB = 0;
  bool fwd_x3 = false;            // the last forward wrote SG (X3 chain)
  // n_skip / n_post that are not multiples of 4 (par/arch2.json: 8 / 6) run padded to the
  // next multiple of 4 inside the plan (Cs, Cp): the head weights are copied into zero-padded
  // images each step (zero rows/columns keep the padded channels at exactly 0 through relu and
  // every product) and the head gradients are copied back out of padded buffers.
  int Cs_ref = 0, Cp_ref = 0;
  size_t oPADP = 0, oPADG = 0;
  int ctrace_blk = -1;            // LBWN_CHAIN_TRACE=<block>: chain cycle stamps (debug)
  size_t oGCTAB, oGCD, oGCPART, oLCACT[8], oCOND, oDVALL, oLCCAT, oDLCCAT, oDLC[2];
  size_t oLCCAT3 = 0;   // LCcat pre-split into bf16 planes (dlc's B; 0 = not used: K % 32 != 0)
  size_t oTGID = 0;              // GC + chain: per-tile uniform voice id (lbwn_gc_tile_sum_launch)
  // Residual-stack weight gradients outside the backward chain (LBWN_BWD_WGRAD=1, round 6): the
  // chain exports DV (oDVALL, k-blocked) and G = dx_{l+1} rows (oGX [L][m32(M)][32]);
  // layer_wgrad_kernel sums them per layer into the slab (oGCS: GC per-tile dv sums)
  bool wg_out = false;
  size_t oGX = 0, oGCS = 0;
  // in-chain LC (bf16-split forward chain): L split LC images; COND is then computed only when a
  // backward path needs it (cond_valid: this step's COND is in the workspace)
  size_t oLCX = 0;
  bool cond_valid = false;
  int split_dlc, split_dlcx, split_dlct, split_up[8];
  size_t oSPLIT_AUX = 0;         // split-K workspace of the aux2 stream (LC / GC grads beside dSKIP)
  bool up_fused = false;         // LC upsample as one fused launch per direction (cond.hip)
  int dlc_parts = 1;             // split-K partials the last dlc GEMM left for the fused upsample backward
  const float* dlc_spl = nullptr;   // ... in this split-K workspace (checked by lc_upsample_bwd)
  bool up_fused_bwd = false;     // ... for the backward (<= 256 mel frames; else per-stage GEMMs)
  size_t oUPPART = 0;            // its per-frame filter-gradient partials
  size_t total;
  long x_layer_stride;  // floats
  int split_post2, split_post1, split_skip;
  long split_floats;
  int nblk;                      // layer-bwd blocks = slab partials per layer
  bool chain = false;            // persistent layer-chain kernels (n_res = n_dil = 32)
  int chain_grid = 0;            // resident blocks for the chain (set on first use)
  int fwd_grid = 0;              // ... for the forward chain (its tile: lbwn_chain_fwd_tile(fwd_nw))
  // chain forms (LBWN_CHAIN_TILE = <fwd>[:<bwd>] at plan creation, each 128 / 64 / w32; default
  // 128): 0 = 32-position waves on 128-position tiles (chain_fwd_kernel / chain_bwd_x3_kernel),
  // 8 / 4 = 16-position waves on 128- / 64-position tiles (chain_fwd16_kernel / chain_bwd16_kernel)
  int fwd_nw = 8, bwd_nw = 8;
  int bwd_grid = 0;
  // Backward side stream (chain plans): the head weight gradients (dPOST2, dPOST1) run on the
  // main stream before the chain; dSKIP follows the chain on the main stream while `aux2` runs
  // the HBM-bound slab reduction and dPRE scatter beside it.  A chain block takes a whole CU's
  // LDS, so nothing co-resides with the chains.
  bool overlap = false;
  hipStream_t aux2 = nullptr;
  hipEvent_t ev_chain = nullptr, ev_join2 = nullptr;
  hipEvent_t ev_fwd_fork = nullptr, ev_fwd_up = nullptr;   // forward: LC upsample on aux2
  hipEvent_t ev_upb = nullptr;   // backward: the upsample's per-frame pass done (main) -> its sum (aux2)
  hipEvent_t ev_dlc = nullptr;   // backward (dlc over more than one round of blocks): dlc done -> aux2
  bool up_forked = false;        // this forward launched the fused upsample on aux2
  bool bwd_chain_event = false;  // the last backward recorded ev_chain (lbwn_plan_stream_wait)
  bool bwd_side_event = false;   // ... and ev_join2 at the end of its side-stream work
  // the bias gradients' final column sums on aux2 beside dPOST2 / dPOST1 (a 41-VGPR kernel that
  // fits beside their blocks), joined before the backward chain: C2 -7 us per step, C4 neutral
  // (profiles/r06_ab_colsum_side.txt); LBWN_COLSUM_SIDE=0 (plan creation) keeps them in line
  bool colsum_side = true;
  hipEvent_t ev_cs = nullptr, ev_cs_done = nullptr;
  bool wpk_valid = false;        // the f32 layer images were packed this step
  // Weights pre-split into bf16 planes once per step for the bf16-split GEMMs (gemm.hip):
  // [W3_SKIP_F] SKIPcat as skip-fwd B, [W3_POST1_F] POST1 as post1-fwd B, [W3_POST2_F] POST2 as
  // post2-fwd B, [W3_POST2_B] POST2ᵀ as dH1 B, [W3_POST1_B] POST1ᵀ as dS B, [W3_SKIP_B]
  // SKIPcatᵀ as dZ B.  Offset 0 = not used (K % 32 != 0).
  size_t oW3[6] = {0, 0, 0, 0, 0, 0};
  ~lbwn_plan() {
    if (aux2) (void)hipStreamDestroy(aux2);
    if (ev_chain) (void)hipEventDestroy(ev_chain);
    if (ev_fwd_fork) (void)hipEventDestroy(ev_fwd_fork);
    if (ev_fwd_up) (void)hipEventDestroy(ev_fwd_up);
    if (ev_upb) (void)hipEventDestroy(ev_upb);
    if (ev_dlc) (void)hipEventDestroy(ev_dlc);
    if (ev_join2) (void)hipEventDestroy(ev_join2);
    if (ev_cs) (void)hipEventDestroy(ev_cs);
    if (ev_cs_done) (void)hipEventDestroy(ev_cs_done);
  }
  // one-shot event probe
  char probe[32];
  hipEvent_t probe_start, probe_stop;
};

namespace {
enum { W3_SKIP_F, W3_POST1_F, W3_POST2_F, W3_POST2_B, W3_POST1_B, W3_SKIP_B };
// (rows = N of the product, K, trans, W's row stride) of each pre-split weight
struct W3Shape { int rows, K, trans, ldw; };
W3Shape w3_shape(const lbwn_plan* p, int i) {
  const int ldz = p->L * p->Cd;
  switch (i) {
    case W3_SKIP_F: return {p->Cs, ldz, 1, p->Cs};
    case W3_POST1_F: return {p->Cp, p->Cs, 1, p->Cp};
    case W3_POST2_F: return {p->Q, p->Cp, 1, p->Q};
    case W3_POST2_B: return {p->Cp, p->Q, 0, p->Q};
    case W3_POST1_B: return {p->Cs, p->Cp, 0, p->Cp};
    default: return {ldz, p->Cs, 0, p->Cs};
  }
}

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

int lbwn_plan_stream_wait(lbwn_plan* p, const char* point, void* stream, int* waited) {
  LBWN_REQUIRE(p && point && waited, "plan_stream_wait: null argument");
  *waited = 0;
  if (!strcmp(point, "head_grads")) {
    // ev_chain: recorded on the main stream right after the backward chain launch, behind the
    // head weight-gradient GEMMs and the bias column sums (padded heads copy theirs out at the end)
    if (p->bwd_chain_event && !p->oPADG) {
      LBWN_HIP(hipStreamWaitEvent((hipStream_t)stream, p->ev_chain, 0));
      *waited = 1;
    }
    return 0;
  }
  if (!strcmp(point, "side_grads")) {
    // ev_join2: recorded on the side stream after its last gradient kernel (dPRE, the slab
    // reduction of SIG/GATE/RES and their biases, the GC table grads; for LC plans also after
    // the upsample's frame sum), while dSKIP may still run on the main stream
    if (p->bwd_side_event) {
      LBWN_HIP(hipStreamWaitEvent((hipStream_t)stream, p->ev_join2, 0));
      *waited = 1;
    }
    return 0;
  }
  LBWN_REQUIRE(false, "plan_stream_wait: unknown point '%s'", point);
  return 0;
}

namespace {

size_t carve(size_t& cur, size_t bytes) {
  size_t o = cur;
  cur += (bytes + 255) / 256 * 256;
  return o;
}

// rows of the SG buffer: whole 32-row blocks (sg_off in layer.hip)
static long m32(long M) { return (M + 31) / 32 * 32; }

// Split-K for the weight-gradient GEMMs (K = B·T positions).  One 4-wave block per CU
// leaves the MFMA pipe latency-exposed, so aim for ~4 resident blocks per CU (1024 blocks)
// with the slab traffic capped at 64 MB.
int pick_split(int M, int N, long K) {
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  const long slab_cap = std::max<long>(1, (64L << 20) / (4L * M * N));
  // one wave of 2-blocks-per-CU slots (512): more splits only add slab traffic (dPOST1 at 64
  // splits wrote 67 MB of slabs for 134 MB of operands, profiles/pmc_traffic.json)
  const long s = std::max<long>(1, std::min<long>({512 / tiles, K / 512, slab_cap}));
  return (int)s;
}

template <typename T>
T* at(void* ws, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}

}  // namespace

namespace {
// padded head images: SKIP [L·Cd][Cs] | SKIP_BIAS [L][Cs] | POST1 [Cs][Cp] | POST1_BIAS [Cp] | POST2 [Cp][Q]
size_t head_pad_floats(const lbwn_plan* p) {
  const size_t L = p->L, Cd = p->Cd, Cs = p->Cs, Cp = p->Cp, Q = p->Q;
  return L * Cd * Cs + L * Cs + Cs * Cp + Cp + Cp * Q + 5 * 64;
}
struct HeadPad { float *skip, *skip_b, *post1, *post1_b, *post2; };
HeadPad head_pad_layout(const lbwn_plan* p, float* base) {
  auto up = [](size_t n) { return (n + 63) / 64 * 64; };   // 256-B aligned pieces
  const size_t L = p->L, Cd = p->Cd, Cs = p->Cs, Cp = p->Cp, Q = p->Q;
  HeadPad h;
  h.skip = base;
  h.skip_b = h.skip + up(L * Cd * Cs);
  h.post1 = h.skip_b + up(L * Cs);
  h.post1_b = h.post1 + up(Cs * Cp);
  h.post2 = h.post1_b + up(Cp);
  return h;
}
// rows x cols (reference widths) <-> the same block at padded row widths
int copy2d(float* dst, size_t dld, const float* src, size_t sld, size_t cols, size_t rows, hipStream_t st) {
  if (!src || !dst) return 0;
  LBWN_HIP(hipMemcpy2DAsync(dst, dld * 4, src, sld * 4, cols * 4, rows, hipMemcpyDeviceToDevice, st));
  return 0;
}
// P (reference layouts) -> zero-padded images; returns the params struct pointing at them
int head_pad_params(const lbwn_plan* p, const lbwn_params* P, void* ws, lbwn_params& out, bool copy,
                    hipStream_t st) {
  out = *P;
  if (!p->oPADP) return 0;
  HeadPad h = head_pad_layout(p, reinterpret_cast<float*>(static_cast<char*>(ws) + p->oPADP));
  const size_t L = p->L, Cd = p->Cd, Cs = p->Cs, Cp = p->Cp, Q = p->Q, cs = p->Cs_ref, cp = p->Cp_ref;
  if (copy) {
    if (int e = lbwn_zero_launch(h.skip, sizeof(float) * head_pad_floats(p), st)) return e;
    int e;
    if ((e = copy2d(h.skip, Cs, P->skip, cs, cs, L * Cd, st))) return e;
    if ((e = copy2d(h.skip_b, Cs, P->skip_b, cs, cs, L, st))) return e;
    if ((e = copy2d(h.post1, Cp, P->post1, cp, cp, cs, st))) return e;
    if ((e = copy2d(h.post1_b, Cp, P->post1_b, cp, cp, 1, st))) return e;
    if ((e = copy2d(h.post2, Q, P->post2, Q, Q, cp, st))) return e;
  }
  out.skip = h.skip; out.post1 = h.post1; out.post2 = h.post2;
  if (P->skip_b) out.skip_b = h.skip_b;
  if (P->post1_b) out.post1_b = h.post1_b;
  return 0;
}
// gradient struct writing into the padded buffers, and the copy back into the caller's
int head_pad_grads(const lbwn_plan* p, const lbwn_params* G, void* ws, lbwn_params& out) {
  out = *G;
  if (!p->oPADG) return 0;
  HeadPad h = head_pad_layout(p, reinterpret_cast<float*>(static_cast<char*>(ws) + p->oPADG));
  out.skip = h.skip; out.post1 = h.post1; out.post2 = h.post2;
  if (G->skip_b) out.skip_b = h.skip_b;
  if (G->post1_b) out.post1_b = h.post1_b;
  return 0;
}
int head_unpad_grads(const lbwn_plan* p, const lbwn_params* G, void* ws, hipStream_t st) {
  if (!p->oPADG) return 0;
  HeadPad h = head_pad_layout(p, reinterpret_cast<float*>(static_cast<char*>(ws) + p->oPADG));
  const size_t L = p->L, Cd = p->Cd, Cs = p->Cs, Cp = p->Cp, Q = p->Q, cs = p->Cs_ref, cp = p->Cp_ref;
  int e;
  if ((e = copy2d(G->skip, cs, h.skip, Cs, cs, L * Cd, st))) return e;
  if (G->skip_b && (e = copy2d(G->skip_b, cs, h.skip_b, Cs, cs, L, st))) return e;
  if ((e = copy2d(G->post1, cp, h.post1, Cp, cp, cs, st))) return e;
  if (G->post1_b && (e = copy2d(G->post1_b, cp, h.post1_b, Cp, cp, 1, st))) return e;
  if ((e = copy2d(G->post2, Q, h.post2, Q, Q, cp, st))) return e;
  return 0;
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
  LBWN_REQUIRE(a->n_skip >= 1 && a->n_post >= 1 && a->n_quant % 4 == 0,
               "plan: n_skip/n_post >= 1 and n_quant a multiple of 4 required");
  LBWN_REQUIRE(B >= 1 && T >= 2, "plan: batch_sz >= 1 and slice_sz >= 2 required");
  LBWN_REQUIRE(a->n_gc_embed >= 0 && (a->n_gc_embed == 0 || a->n_gc_category >= 1),
               "plan: GC needs n_gc_category >= 1");
  LBWN_REQUIRE(a->n_gc_embed <= 32, "plan: n_gc_embed > 32 not supported");
  int hop = 1;
  if (a->n_lc_out > 0) {
    LBWN_REQUIRE(a->n_lc_upsample >= 1 && a->n_lc_upsample <= 8, "plan: LC needs 1..8 upsample stages");
    for (int i = 0; i < a->n_lc_upsample; ++i) {
      LBWN_REQUIRE(a->lc_upsample[i] >= 1, "plan: bad lc_upsample stride");
      hop *= a->lc_upsample[i];
    }
    LBWN_REQUIRE(T % hop == 0, "plan: slice_sz %d is not a multiple of the mel hop %d", T, hop);
    LBWN_REQUIRE(a->n_lc_in % 4 == 0 && a->n_lc_out % 4 == 0, "plan: n_lc_in/n_lc_out must be multiples of 4");
  }
  // chain forms (lbwn_plan::fwd_nw): default 16-position waves on 128-position tiles (same-box A/B,
  // profiles/r04_ab_chain16_tiles.txt: arch3 forward chain 278 -> 241 us, backward 492 -> 419 us)
  int fwd_nw = 8, bwd_nw = 8;
  {
    const char* tv = getenv("LBWN_CHAIN_TILE");
    auto form = [](const char* v, size_t n, int* nw) {
      if (n == 2 && !strncmp(v, "64", 2)) *nw = 4;
      else if (n == 3 && !strncmp(v, "128", 3)) *nw = 8;
      else if (n == 3 && !strncmp(v, "w32", 3)) *nw = 0;
      else return false;
      return true;
    };
    if (tv && tv[0]) {
      const char* colon = strchr(tv, ':');
      const size_t nf = colon ? (size_t)(colon - tv) : strlen(tv);
      bool ok = form(tv, nf, &fwd_nw);
      if (ok) ok = colon ? form(colon + 1, strlen(colon + 1), &bwd_nw) : form(tv, nf, &bwd_nw);
      LBWN_REQUIRE(ok, "LBWN_CHAIN_TILE must be <fwd>[:<bwd>] with each 128, 64 or w32 (got '%s')", tv);
    }
  }
  lbwn_plan* p = new (std::nothrow) lbwn_plan();
  LBWN_REQUIRE(p, "plan: out of host memory");
  p->fwd_nw = fwd_nw;
  p->bwd_nw = bwd_nw;
  p->a = *a;
  p->B = B;
  p->T = T;
  p->nbl = a->n_block_layers;
  p->L = a->n_blocks * a->n_block_layers;
  p->H = 1 << (a->n_block_layers - 1);
  p->Cr = a->n_res;
  p->Cd = a->n_dil;
  p->Cs_ref = a->n_skip;
  p->Cp_ref = a->n_post;
  p->Cs = (a->n_skip + 3) / 4 * 4;
  p->Cp = (a->n_post + 3) / 4 * 4;
  p->Q = a->n_quant;
  p->M = (long)B * T;
  p->Ge = a->n_gc_embed;
  p->ncat1 = a->n_gc_embed > 0 ? a->n_gc_category + 1 : 0;
  p->Lo = a->n_lc_out;
  {  // XCD-grouped chain tile walk (layer.hip chain_first): on for LC archs only.  Same box, two
     // rounds (profiles/r04_ab_chain_xcd_lc.txt): arch5 B=8 2.748-2.761 vs 2.777-2.779 ms (the
     // LC products read the k-blocked DV export the chain wrote), arch3 B=8 2.101-2.104 vs
     // 2.082-2.091 (its forward chain 248 vs 239-240 us; profiles/r04_ab_handoff_xcd.txt).
     // LBWN_CHAIN_XCD=0 / 1 overrides.  Placement only: bitwise the same results.
    const char* xv = getenv("LBWN_CHAIN_XCD");
    p->chain_xcd = xv ? (strcmp(xv, "1") == 0) : (p->Lo > 0);
    // dZ's 2-D XCD tile blocking (profiles/r04_ab_dz_xcd.txt: time-neutral, 490 -> 460 MB per
    // launch); LBWN_DZ_XCD=0 keeps the 1-D remap.  Placement only: bitwise the same results.
    const char* dv = getenv("LBWN_DZ_XCD");
    p->dz_xcd2d = (dv && dv[0] == '0') ? 0 : 1;
    // weight gradients of the residual stack: inside the backward chain (0) or by
    // layer_wgrad_kernel over the chain's exports (1; 16-position backward on 128-position tiles)
    const char* mv = getenv("LBWN_GEMM_MBITS");
    p->mbits_ok = !(mv && mv[0] == '0');
    const char* wv = getenv("LBWN_BWD_WGRAD");
    p->wg_out = (wv && wv[0] == '1') && bwd_nw == 8;
    const char* cv = getenv("LBWN_COLSUM_SIDE");
    p->colsum_side = !(cv && cv[0] == '0');
  }
  p->Li = a->n_lc_in;
  p->nup = a->n_lc_out > 0 ? a->n_lc_upsample : 0;
  p->hop = hop;
  for (int i = 0; i < 8; ++i) p->up[i] = i < p->nup ? a->lc_upsample[i] : 1;
  const long M = p->M;
  const int L = p->L;
  p->x_layer_stride = (long)B * (p->H + T) * p->Cr;
  // keep every x row 16-B aligned for the vector path
  p->x_layer_stride = (p->x_layer_stride + 3) / 4 * 4;
  const long ldz = (long)L * p->Cd;
  p->split_post2 = pick_split(p->Cp, p->Q, M);
  p->split_post1 = pick_split(p->Cs, p->Cp, M);
  p->split_skip = pick_split(L * p->Cd, p->Cs, M);
  p->split_floats = std::max({(long)p->split_post2 * p->Cp * p->Q, (long)p->split_post1 * p->Cs * p->Cp,
                              (long)p->split_skip * ldz * p->Cs});
  if (p->Lo > 0) {
    p->split_dlc = pick_split(p->Lo, 2 * L * p->Cd, M);
    p->split_floats = std::max(p->split_floats, (long)p->split_dlc * p->Lo * 2 * L * p->Cd);
    // dlc = DV·LCcatᵀ (M × n_lc_out, K = L·2Cd): 256-row tiles, one N tile; split K until the
    // grid has ~one block per CU (it ran on 128 blocks of 256 CUs at B = 8; it runs beside dLCcat,
    // so 512 blocks measured slower: C5 per GPU 3.11 -> 3.06 ms at 256 blocks, same box)
    const long dtiles = (M + 255) / 256 * ((p->Lo + 127) / 128);
    p->split_dlcx = (int)std::max<long>(1, std::min<long>(256 / std::max<long>(1, dtiles), (2L * L * p->Cd) / 256));
    p->split_floats = std::max(p->split_floats, (long)p->split_dlcx * M * p->Lo);
    // dLCcat as DVᵀ·lc (the AMN form, lc_wgrad): ceil(L·2Cd / 256) row tiles, K = M split to
    // about one block per CU
    const long ttiles = (2L * L * p->Cd + 255) / 256;
    p->split_dlct = (int)std::max<long>(1, std::min<long>(256 / ttiles, M / 256));
    p->split_floats = std::max(p->split_floats, (long)p->split_dlct * 2 * L * p->Cd * p->Lo);
    long rows = (long)B * (T / hop);
    for (int i = 0; i < p->nup; ++i) {
      const int I = i == 0 ? p->Li : p->Lo;
      p->split_up[i] = pick_split(p->up[i] * p->Lo, I, rows);
      p->split_floats = std::max(p->split_floats, (long)p->split_up[i] * p->up[i] * p->Lo * I);
      rows *= p->up[i];
    }
  }
  const int nblk = lbwn_layer_bwd_grid(B, T);
  p->nblk = nblk;
  size_t cur = 0;
  p->oX = carve(cur, sizeof(float) * (size_t)p->x_layer_stride * L);
  p->oZ = carve(cur, sizeof(float) * (size_t)M * ldz);
  p->oS = carve(cur, sizeof(float) * (size_t)M * p->Cs);
  p->oR2 = carve(cur, sizeof(float) * (size_t)M * p->Cp);
  p->oLOG = carve(cur, sizeof(float) * (size_t)M * p->Q);
  p->oDH = carve(cur, sizeof(float) * (size_t)M * p->Cp);
  p->oDS = carve(cur, sizeof(float) * (size_t)M * p->Cs);
  p->oDZ = carve(cur, sizeof(float) * (size_t)m32(M) * ldz);   // chain order (x3 chain): whole 32-row blocks
  for (int i = 0; i < 2; ++i) {
    p->oGA[i] = carve(cur, sizeof(float) * (size_t)M * p->Cr);
    p->oGC0[i] = carve(cur, sizeof(float) * (size_t)M * p->Cr);
  }
  const int ntiles = B * ((T + 63) / 64);   // the finest chain tile: any backward form fits
  p->oSLAB = carve(cur, sizeof(float) * (size_t)L * std::max(nblk, ntiles) * lbwn_layer_slab_stride());
  p->oSPLIT = carve(cur, sizeof(float) * (size_t)p->split_floats);
  p->oSPLIT2 = carve(cur, sizeof(float) * (size_t)lbwn_pre_grad_ws_floats(p->Q, p->Cr));   // dPRE partials
  // three column sums at once in the backward (dlogits, dH1, dS)
  p->oCOLS = carve(cur, sizeof(float) * 3 * (size_t)lbwn_colsum_ws_floats((int)M, std::max({p->Cs, p->Cp, p->Q, p->Cr})));
  // dH1 / dS column partials from the GEMM epilogues (bias gradients of POST1 / SKIP)
  p->oCPART = carve(cur, sizeof(float) * (size_t)lbwn_colpart_parts(M) * (p->Cp + p->Cs));
  // [status (16 B) | forward hand-off flags | backward hand-off flags], zeroed by ONE memset per
  // step (each flag block padded to 16 B)
  // one flag per 16-position wave of a tile (the 16-position chains' per-wave hand-offs; the
  // 32-position forms use one per 128-position tile), so any form fits: ceil(T/TP)·NW <= T/16 + 8
  p->nflag_bytes = (sizeof(unsigned) * (size_t)B * ((T + 15) / 16 + 8) + 15) / 16 * 16;
  p->oSTATUS = carve(cur, 16 + 2 * p->nflag_bytes);
  p->oFLAGS = p->oSTATUS + 16;
  {
    const char* ct = getenv("LBWN_CHAIN_TRACE");
    p->ctrace_blk = ct ? atoi(ct) : -1;
    p->oCTRACE = carve(cur, 8 * 2 * 16 * (size_t)L);   // [fwd, bwd][L][16]
  }
  const char* nc = getenv("LBWN_NO_CHAIN");
  p->chain = p->Cr == 32 && p->Cd == 32 && !(nc && nc[0] == '1');
  // the 16-position backward chain addresses its per-layer dZ / σ / z rows with 32-bit lane offsets
  // (chain_bwd16_kernel load_regs): refuse here, not at the first backward after a whole forward
  if (p->chain && bwd_nw && (long)M * ldz * 4 >= 0x7fffffffL) {
    delete p;
    LBWN_REQUIRE(false, "plan: B*T*n_layers*n_dil*4 = %ld bytes of z rows is past the backward chain's 2 GiB lane "
                        "offsets (LBWN_NO_CHAIN=1 runs the per-layer kernels)", (long)M * ldz * 4);
  }
  p->oOCG = p->chain ? carve(cur, sizeof(float) * (size_t)L * M * 32) : 0;
  p->oSG = p->chain ? carve(cur, sizeof(float) * (size_t)L * m32(M) * 32) : 0;   // sg_off: whole 32-row blocks
  p->overlap = p->chain;
  if (p->overlap && (p->Lo > 0 || p->Ge > 0)) p->oSPLIT_AUX = carve(cur, sizeof(float) * (size_t)p->split_floats);
  {  // conditioning
    const size_t f = sizeof(float);
    const long ncond = 2L * L * p->Cd;
    p->oGCTAB = p->Ge ? carve(cur, f * (size_t)L * p->ncat1 * 2 * p->Cd) : 0;
    p->oGCD = p->Ge ? carve(cur, f * (size_t)L * p->ncat1 * 2 * p->Cd) : 0;
    p->oTGID = p->Ge ? carve(cur, sizeof(int) * (size_t)B * ((T + 63) / 64)) : 0;
    p->oGCPART = p->Ge ? carve(cur, f * (size_t)lbwn_gc_part_floats(L, p->Ge, p->Cd)) : 0;
    long rows = (long)B * (T / hop);
    for (int i = 0; i < 8; ++i) {
      p->oLCACT[i] = 0;
      if (i < p->nup) {
        rows *= p->up[i];
        p->oLCACT[i] = carve(cur, f * (size_t)rows * p->Lo);
      }
    }
    p->oCOND = p->Lo ? carve(cur, f * (size_t)M * ncond) : 0;
    p->up_fused = p->Lo > 0 && lbwn_lc_up_fused_ok(p->nup, p->up, p->Li, p->Lo);
    // The fused backward runs one block per mel frame at one block per CU: past one round of
    // frames the per-stage GEMMs win (same box, profiles/r04_ab_lc_upsample.txt: arch5 B=8, 128
    // frames, fused 2.817-2.829 ms vs GEMMs 2.955-2.957; B=32, 512 frames, fused 10.67-10.68 vs
    // 10.56-10.57)
    p->up_fused_bwd = p->up_fused && M / hop <= 256;
    if (p->up_fused) p->oUPPART = carve(cur, f * (size_t)lbwn_lc_up_part_floats(p->nup, p->up, p->Li, p->Lo, (int)(M / hop)));
    // rows or [2L][m32(M)][32]; also the export form's DV
    p->oDVALL = (p->Lo || (p->chain && p->wg_out)) ? carve(cur, f * (size_t)m32(M) * ncond) : 0;
    if (p->chain && p->wg_out) {
      p->oGX = carve(cur, f * (size_t)L * m32(M) * 32);
      p->oGCS = p->Ge ? carve(cur, f * (size_t)L * B * ((T + 127) / 128) * 64) : 0;
    }
    p->oLCCAT = p->Lo ? carve(cur, f * (size_t)p->Lo * ncond) : 0;
    if (p->Lo && ncond % 32 == 0)
      p->oLCCAT3 = carve(cur, sizeof(unsigned short) * lbwn_split_planes_elems(p->Lo, (int)ncond));
    p->oDLCCAT = p->Lo ? carve(cur, f * (size_t)p->Lo * ncond) : 0;
    for (int i = 0; i < 2; ++i) p->oDLC[i] = p->Lo ? carve(cur, f * (size_t)M * std::max(p->Lo, p->Li)) : 0;
  }
  for (int i = 0; i < 6; ++i) {
    const W3Shape w = w3_shape(p, i);
    if (w.K % 32 == 0) p->oW3[i] = carve(cur, 2 * lbwn_split_planes_elems(w.rows, w.K));
  }
  if (p->chain && p->Lo > 0 && lbwn_lc_in_chain_ok(p->Lo))
    p->oLCX = carve(cur, 2 * (size_t)L * std::max(lbwn_lc_image_x3_elems(), lbwn_lc_image16_elems()));
  p->oMBS = carve(cur, 8 * (size_t)lbwn_gemm_mbits_words(M, p->Cs));
  p->oMBR = carve(cur, 8 * (size_t)lbwn_gemm_mbits_words(M, p->Cp));
  p->oHEADP = carve(cur, sizeof(float) * 3 * 2048);
  p->oBSUM = carve(cur, sizeof(float) * (size_t)p->Cs);
  p->oWPK = carve(cur, sizeof(float) * (size_t)L * lbwn_layer_image_floats());
  p->oWPKX = carve(cur, 2 * (size_t)L * lbwn_layer_image_x3_elems());
  p->oWPKB = carve(cur, sizeof(float) * (size_t)L * lbwn_layer_image_bx3_floats());
  if (p->Cs != p->Cs_ref || p->Cp != p->Cp_ref) {
    const size_t hp = head_pad_floats(p);
    p->oPADP = carve(cur, sizeof(float) * hp);
    p->oPADG = carve(cur, sizeof(float) * hp);
  }
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
  else if (!strcmp(name, "status")) { *off = p->oSTATUS; *bytes = 16; }
  else if (!strcmp(name, "ctrace")) { *off = p->oCTRACE; *bytes = 8 * 2 * 16 * (size_t)p->a.n_blocks * p->a.n_block_layers; }
  else if (!strcmp(name, "dh")) { *off = p->oDH; *bytes = f * M * p->Cp; }
  else if (!strcmp(name, "ds")) { *off = p->oDS; *bytes = f * M * p->Cs; }
  else if (!strcmp(name, "dz")) { *off = p->oDZ; *bytes = f * M * p->L * p->Cd; }
  else if (!strcmp(name, "cond") && p->Lo) { *off = p->oCOND; *bytes = f * M * 2 * p->L * p->Cd; }
  else if (!strcmp(name, "dvall") && p->Lo) {   // rows [M][L·2Cd], or k-blocked [2L][m32(M)][32] (dv_blk)
    *off = p->oDVALL;
    *bytes = f * (p->dv_blk ? (size_t)m32(p->M) : M) * 2 * p->L * p->Cd;
  }
  else if (!strcmp(name, "gctab") && p->Ge) { *off = p->oGCTAB; *bytes = f * p->ncat1 * 2 * p->L * p->Cd; }
  else if (!strcmp(name, "gcd") && p->Ge) { *off = p->oGCD; *bytes = f * p->ncat1 * 2 * p->L * p->Cd; }
  else LBWN_REQUIRE(false, "plan_tensor: unknown tensor '%s'", name);
  return 0;
}
size_t lbwn_plan_workspace_bytes(const lbwn_plan* p) { return p ? p->total : 0; }

// pre-split planes of weight i when the bf16-split GEMM is active, else null
static const unsigned short* w3(const lbwn_plan* p, void* ws, int i) {
  return (p->oW3[i] && lbwn_gemm_mode() == 1) ? reinterpret_cast<const unsigned short*>(static_cast<char*>(ws) + p->oW3[i])
                                              : nullptr;
}

static lbwn_gemm_args gemm0() {
  lbwn_gemm_args g;
  memset(&g, 0, sizeof(g));
  return g;
}

namespace {

// Device facts needed at first launch (not at plan creation, which must work without a GPU).
int ensure_device(lbwn_plan* p) {
  if (p->chain_grid) return 0;
  // chain grid: at most one block per CU, so every block of a round is resident
  int dev = 0, ncu = 0;
  LBWN_HIP(hipGetDevice(&dev));
  LBWN_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  p->ncu = ncu;
  const int ntiles = p->B * ((p->T + LBWN_LAYER_POS - 1) / LBWN_LAYER_POS);
  p->chain_grid = std::max(1, std::min(ntiles, ncu));
  const int tpf = lbwn_chain_fwd_tile(p->fwd_nw);
  p->fwd_grid = std::max(1, std::min(p->B * ((p->T + tpf - 1) / tpf), ncu));
  const int tpb = lbwn_chain_fwd_tile(p->bwd_nw);
  p->bwd_grid = std::max(1, std::min(p->B * ((p->T + tpb - 1) / tpb), ncu));
  if (p->overlap) {
    int least = 0, greatest = 0;
    LBWN_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    LBWN_HIP(hipStreamCreateWithPriority(&p->aux2, hipStreamNonBlocking, greatest));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_chain, hipEventDisableTiming));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_join2, hipEventDisableTiming));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_fwd_fork, hipEventDisableTiming));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_fwd_up, hipEventDisableTiming));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_upb, hipEventDisableTiming));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_dlc, hipEventDisableTiming));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_cs, hipEventDisableTiming));
    LBWN_HIP(hipEventCreateWithFlags(&p->ev_cs_done, hipEventDisableTiming));
  }
  return 0;
}

lbwn_layer_args layer_base(const lbwn_plan* p, const lbwn_params* P, const float* WPK, const int* ids, int l) {
  const int Cr = p->Cr, Cd = p->Cd;
  lbwn_layer_args a;
  memset(&a, 0, sizeof(a));
  a.w_sig = P->sig + (long)l * 2 * Cr * Cd;
  a.w_gate = P->gate + (long)l * 2 * Cr * Cd;
  a.b_sig = P->sig_b ? P->sig_b + (long)l * Cd : nullptr;
  a.b_gate = P->gate_b ? P->gate_b + (long)l * Cd : nullptr;
  a.w_res = P->res + (long)l * Cd * Cr;
  a.b_res = P->res_b ? P->res_b + (long)l * Cr : nullptr;
  a.wpack = WPK + (long)l * lbwn_layer_image_floats();
  a.ids = ids;
  a.B = p->B; a.T = p->T; a.H = p->H; a.d = 1 << (l % p->nbl); a.Cr = Cr; a.Cd = Cd;
  return a;
}

}  // namespace

namespace {

// Conditioning operands of the layer stack (tmodel.py:105-114, :150-160)
struct Cond {
  const float* gc_tab = nullptr; long gc_ld = 0;   // GCTAB [ncat+1][L·2Cd]
  const float* cond = nullptr; long ldcond = 0;     // COND [M][L·2Cd]
  float* gc_dtab = nullptr;                         // backward: GCD
  float* dv_out = nullptr;                          // backward: DVALL
  void apply(lbwn_layer_args& a, int l) const {
    a.gc_tab = gc_tab ? gc_tab + (long)l * 2 * a.Cd : nullptr;
    a.gc_dtab = gc_dtab ? gc_dtab + (long)l * 2 * a.Cd : nullptr;
    a.gc_ld = gc_ld;
    a.cond = cond ? cond + (long)l * 2 * a.Cd : nullptr;
    a.ldcond = ldcond;
    a.dv_out = dv_out ? dv_out + (long)l * 2 * a.Cd : nullptr;
    a.lddv = ldcond;
  }
};

// the forward chain computes the LC term itself (bf16-split chain, 64 < n_lc_out <= 80)
bool lc_in_chain(const lbwn_plan* p) { return p->oLCX && p->chain && lbwn_gemm_mode() == 1; }

// COND = lc·LCcat [M][L·2Cd]: every layer's LC term (tmodel.py:155-160) as ONE GEMM, for the paths
// that read it (f32 chains, per-layer kernels)
int cond_project(lbwn_plan* p, const lbwn_params* P, void* ws, hipStream_t st) {
  int e;
  const long ncond = 2L * p->L * p->Cd;
  float* cat = at<float>(ws, p->oLCCAT);
  if ((e = lbwn_lc_pack_launch(cat, P->lc_sig, P->lc_gate, p->L, p->Lo, p->Cd, 1, st))) return e;
  lbwn_gemm_args g = gemm0();
  g.A = at<float>(ws, p->oLCACT[p->nup - 1]); g.lda = p->Lo; g.B = cat; g.ldb = ncond;
  g.C = at<float>(ws, p->oCOND); g.ldc = ncond;
  g.M = (int)p->M; g.N = (int)ncond; g.K = p->Lo;
  Probe(p, st, "lc_cond");
  if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
  Probe::end(p, st, "lc_cond");
  p->cond_valid = true;
  return 0;
}

// GC table and the LC term: upsample (4× conv1d_transpose k = s, tmodel.py:68-83, each a GEMM
// against the [s][O][I] filter read as k-contiguous), then COND = lc·LCcat unless the forward
// chain computes the LC term itself.
int cond_forward(lbwn_plan* p, const lbwn_params* P, void* ws, const float* mel, Cond& c, hipStream_t st) {
  int e;
  const int L = p->L, Cd = p->Cd;
  if (p->Ge > 0) {
    float* tab = at<float>(ws, p->oGCTAB);
    if ((e = lbwn_gc_table_launch(P->gc_embed, P->gc_sig, P->gc_gate, tab, L, p->ncat1, p->Ge, Cd, st))) return e;
    c.gc_tab = tab;
    c.gc_ld = 2L * L * Cd;
  }
  if (p->Lo > 0 && p->up_fused) {
    if (p->up_forked) {   // launched on aux2 at the forward's start; wait for it here
      LBWN_HIP(hipStreamWaitEvent(st, p->ev_fwd_up, 0));
    } else {
      float* act[8];
      for (int i = 0; i < p->nup; ++i) act[i] = at<float>(ws, p->oLCACT[i]);
      Probe(p, st, "lc_up_fwd");
      if ((e = lbwn_lc_up_fwd_launch(p->nup, p->up, p->Li, p->Lo, (int)(p->M / p->hop), mel, P->lc_up, act, st)))
        return e;
      Probe::end(p, st, "lc_up_fwd");
    }
  } else if (p->Lo > 0) {
    const float* in = mel;
    long rows = (long)p->B * (p->T / p->hop);
    int I = p->Li;
    for (int i = 0; i < p->nup; ++i) {
      const int s = p->up[i];
      float* out = at<float>(ws, p->oLCACT[i]);
      lbwn_gemm_args g = gemm0();
      g.A = in; g.lda = I; g.B = P->lc_up[i]; g.ldb = I; g.C = out; g.ldc = (long)s * p->Lo;
      g.M = (int)rows; g.N = s * p->Lo; g.K = I;
      if ((e = lbwn_gemm_launch(g, 1, 1, 1, nullptr, st))) return e;
      in = out;
      rows *= s;
      I = p->Lo;
    }
  }
  if (p->Lo > 0) {
    p->cond_valid = false;
    if (!lc_in_chain(p)) {
      if ((e = cond_project(p, P, ws, st))) return e;
      c.cond = at<float>(ws, p->oCOND);
      c.ldcond = 2L * L * Cd;
    }
  }
  return 0;
}

// After the layer stack: GC weight/table grads from GCD (gc_backward); LC grads from DVALL:
// dLCcat = lcᵀ·DV (lc_wgrad), dlc = DV·LCcatᵀ (lc_dlc), then the upsample stages in reverse
// (lc_upsample_bwd), each a (split-K) GEMM.  The chain plans run them beside dSKIP (engine
// backward); spl is the split-K workspace of the stream they run on.
int gc_backward(lbwn_plan* p, const lbwn_params* P, const lbwn_params* G, void* ws, hipStream_t st) {
  if (p->Ge <= 0) return 0;
  return lbwn_gc_grad_launch(P->gc_embed, P->gc_sig, P->gc_gate, at<float>(ws, p->oGCD), at<float>(ws, p->oGCPART),
                             G->gc_embed, G->gc_sig, G->gc_gate, p->L, p->ncat1, p->Ge, p->Cd, st);
}

int lc_wgrad(lbwn_plan* p, const lbwn_params* G, void* ws, float* spl, hipStream_t st) {
  int e;
  const long ncond = 2L * p->L * p->Cd;
  if (p->dv_blk && lbwn_gemm_mode() == 1 && p->M % 32 == 0 && p->Lo % 4 == 0 && ncond >= 256) {
    // dLCcatᵀ = DVᵀ·lc on the A-in-registers weight-gradient kernel (AMN, 96-column tiles): A = the
    // k-blocked DV export read as 32-row groups (a_gstride), B = the LC rows; C = [L·2Cd][Lo]
    // (the LDS-staged kernel on lcᵀ·DV: C4 569 us)
    lbwn_gemm_args g = gemm0();
    g.A = at<float>(ws, p->oDVALL); g.lda = 32; g.a_gstride = m32(p->M) * 32;
    g.B = at<float>(ws, p->oLCACT[p->nup - 1]); g.ldb = p->Lo;
    g.C = at<float>(ws, p->oDLCCAT); g.ldc = p->Lo;
    g.M = (int)ncond; g.N = p->Lo; g.K = (int)p->M;
    Probe(p, st, "lc_wgrad");
    if ((e = lbwn_gemm_launch(g, 0, 0, p->split_dlct, spl, st))) return e;
    Probe::end(p, st, "lc_wgrad");
    return lbwn_lc_pack_launch(at<float>(ws, p->oDLCCAT), G->lc_sig, G->lc_gate, p->L, p->Lo, p->Cd, 2, st);
  }
  lbwn_gemm_args g = gemm0();
  g.A = at<float>(ws, p->oLCACT[p->nup - 1]); g.lda = p->Lo; g.B = at<float>(ws, p->oDVALL); g.ldb = ncond;
  if (p->dv_blk) { g.ldb = 32; g.b_gstride = m32(p->M) * 32; }
  g.C = at<float>(ws, p->oDLCCAT); g.ldc = ncond;
  g.M = p->Lo; g.N = (int)ncond; g.K = (int)p->M;
  Probe(p, st, "lc_wgrad");
  if ((e = lbwn_gemm_launch(g, 0, 0, p->split_dlc, spl, st))) return e;
  Probe::end(p, st, "lc_wgrad");
  return lbwn_lc_pack_launch(at<float>(ws, p->oDLCCAT), G->lc_sig, G->lc_gate, p->L, p->Lo, p->Cd, 0, st);
}

int lc_dlc(lbwn_plan* p, const lbwn_params* P, void* ws, float* spl, hipStream_t st) {
  int e;
  const long ncond = 2L * p->L * p->Cd;
  // LCcat is packed by the forward's COND projection; an in-chain-LC forward did not run it
  if (!p->cond_valid && (e = lbwn_lc_pack_launch(at<float>(ws, p->oLCCAT), P->lc_sig, P->lc_gate, p->L, p->Lo, p->Cd,
                                                 1, st)))
    return e;
  lbwn_gemm_args g = gemm0();
  g.A = at<float>(ws, p->oDVALL); g.lda = ncond; g.B = at<float>(ws, p->oLCCAT); g.ldb = ncond;
  if (p->dv_blk) { g.lda = 32; g.a_kstride = m32(p->M) * 32; }
  g.C = at<float>(ws, p->oDLC[0]); g.ldc = p->Lo;
  g.M = (int)p->M; g.N = p->Lo; g.K = (int)ncond;
  if (p->oLCCAT3 && lbwn_gemm_mode() == 1) {   // pre-split B: the A-in-registers GEMM (96-column tiles)
    const float* w = g.B;
    const long ld = ncond;
    const int rows = p->Lo, K = (int)ncond, tr = 0;
    unsigned short* o = at<unsigned short>(ws, p->oLCCAT3);
    if ((e = lbwn_split_planes_launch(1, &w, &ld, &rows, &K, &tr, &o, st))) return e;
    g.b3 = o;
  }
  // the fused upsample backward sums dlc's split-K partials as it loads them (no reduce launch
  // between the two on the main stream); the per-stage path reads the reduced dlc
  p->dlc_parts = 1;
  p->dlc_spl = spl;
  if (p->up_fused_bwd) g.splits_deferred = &p->dlc_parts;
  Probe(p, st, "lc_dlc");
  if ((e = lbwn_gemm_launch(g, 1, 1, p->split_dlcx, spl, st))) return e;
  Probe::end(p, st, "lc_dlc");
  return 0;
}

int lc_upsample_bwd(lbwn_plan* p, const lbwn_params* P, const lbwn_params* G, void* ws, const float* mel, float* spl,
                    hipStream_t st, hipStream_t st_sum = nullptr) {
  int e;
  const float* dout = at<float>(ws, p->oDLC[0]);
  if (p->up_fused_bwd) {
    const float* F[8];
    float* act[8];
    for (int i = 0; i < p->nup; ++i) { F[i] = P->lc_up[i]; act[i] = at<float>(ws, p->oLCACT[i]); }
    Probe(p, st, "lc_up_bwd");
    // dlc as the dlc GEMM left it: dlc_parts split-K partials in spl, or the product itself.  The
    // partials live only in that workspace: lc_dlc must have run last on this same spl (no launch
    // that uses spl may sit between the two, on any stream -- the three call sites hold this)
    const bool parts = p->dlc_parts > 1;
    LBWN_REQUIRE(!parts || p->dlc_spl == spl, "lc upsample bwd: dlc's split-K partials are in another workspace");
    e = lbwn_lc_up_bwd_launch(p->nup, p->up, p->Li, p->Lo, (int)(p->M / p->hop), mel, F, act, parts ? spl : dout,
                              at<float>(ws, p->oUPPART), G->lc_up, st, st_sum, p->ev_upb, p->dlc_parts,
                              parts ? p->M * p->Lo : 0);
    Probe::end(p, st, "lc_up_bwd");
    return e;
  }
  long rows = p->M;
  int buf = 0;
  Probe(p, st, "lc_up_bwd");
  for (int i = p->nup - 1; i >= 0; --i) {
    const int s = p->up[i], I = i == 0 ? p->Li : p->Lo;
    rows /= s;  // stage input rows
    const float* in = i == 0 ? mel : at<float>(ws, p->oLCACT[i - 1]);
    // dF_i[(j,o)][i'] = Σ_bt dout[bt][(j,o)] · in[bt][i']
    lbwn_gemm_args g = gemm0();
    g.A = dout; g.lda = (long)s * p->Lo; g.B = in; g.ldb = I; g.C = G->lc_up[i]; g.ldc = I;
    g.M = s * p->Lo; g.N = I; g.K = (int)rows;
    if ((e = lbwn_gemm_launch(g, 0, 0, p->split_up[i], spl, st))) return e;
    if (i == 0) break;  // no gradient into the mel input
    float* din = at<float>(ws, p->oDLC[buf ^ 1]);
    g = gemm0();
    g.A = dout; g.lda = (long)s * p->Lo; g.B = P->lc_up[i]; g.ldb = I; g.C = din; g.ldc = I;
    g.M = (int)rows; g.N = I; g.K = s * p->Lo;
    if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
    dout = din;
    buf ^= 1;
  }
  Probe::end(p, st, "lc_up_bwd");
  return 0;
}

}  // namespace

int lbwn_train_forward(lbwn_plan* p, const lbwn_params* P, void* ws, const int* wav_q, const int* ids,
                       const float* mel, float* save, float* stats, void* stream) {
  LBWN_REQUIRE(p && P && ws && wav_q && ids && save && stats, "train_forward: null argument");
  hipStream_t st = (hipStream_t)stream;
  int e;
  if ((e = ensure_device(p))) return e;
  LBWN_REQUIRE(p->Lo == 0 || mel, "train_forward: LC arch needs the mel input");
  lbwn_params Ppad;
  if ((e = head_pad_params(p, P, ws, Ppad, true, st))) return e;
  P = &Ppad;
  p->fwd_mode = lbwn_gemm_mode();
  // the sticky status word (chain spin timeouts OR their codes in) lives for one step:
  // zeroed here, read by the host after the step (lbwn_plan_tensor "status")
  // (in the fused prologue below when the bf16-split chains run)
  const bool fused_pro = lbwn_gemm_mode() == 1 && p->chain;
  if (!fused_pro && (e = lbwn_zero_launch(at<char>(ws, p->oSTATUS), 16 + 2 * p->nflag_bytes, st))) return e;
  p->bwd_flags_fresh = true;
  // the fused LC upsample depends only on the mel input and the upsample filters: it runs on
  // aux2 beside the weight packs, embedding, GC table and D-sep prepend, joined before the chain
  p->up_forked = false;
  if (p->Lo > 0 && p->up_fused && p->aux2) {
    float* act[8];
    for (int i = 0; i < p->nup; ++i) act[i] = at<float>(ws, p->oLCACT[i]);
    LBWN_HIP(hipEventRecord(p->ev_fwd_fork, st));
    LBWN_HIP(hipStreamWaitEvent(p->aux2, p->ev_fwd_fork, 0));
    if ((e = lbwn_lc_up_fwd_launch(p->nup, p->up, p->Li, p->Lo, (int)(p->M / p->hop), mel, P->lc_up, act, p->aux2)))
      return e;
    LBWN_HIP(hipEventRecord(p->ev_fwd_up, p->aux2));
    p->up_forked = true;
  }
  const int L = p->L, B = p->B, T = p->T, H = p->H, Cr = p->Cr, Cd = p->Cd;
  const long M = p->M, ldz = (long)L * Cd;
  float* X = at<float>(ws, p->oX);
  float* Z = at<float>(ws, p->oZ);
  float* S = at<float>(ws, p->oS);
  float* R2 = at<float>(ws, p->oR2);
  float* LOG = at<float>(ws, p->oLOG);
  float* bsum = at<float>(ws, p->oBSUM);
  // Weight packs (once per step, reused by the backward), in line on the main stream (on a
  // forked side stream the event round trips cost what the overlap hid)
  const bool x3 = lbwn_gemm_mode() == 1;
  hipStream_t pst = st;
  // per-layer weights -> padded f32 LDS images: the per-layer kernels and the f32 chains (the
  // bf16-split chains read their own images below)
  float* WPK = at<float>(ws, p->oWPK);
  p->wpk_valid = !(x3 && p->chain && p->oSG);
  if (p->wpk_valid &&
      (e = lbwn_pack_layers_launch(P->sig, P->gate, P->sig_b, P->gate_b, P->res, P->res_b, WPK, L, Cr, Cd, pst)))
    return e;
  // skip/head weights -> bf16 planes for the split GEMMs, forward and backward, and the split
  // per-layer images of the forward chain
  // ... and the backward chain's split images (dx weights + f32 residual image), one launch
  const bool lcx = lc_in_chain(p);
  const bool bsum_done = x3 && p->chain && P->skip_b;   // summed by the pack (or prologue) launch
  lbwn_prologue_args pa;
  memset(&pa, 0, sizeof(pa));
  if (x3) {
    const float* wsrc[6] = {P->skip, P->post1, P->post2, P->post2, P->post1, P->skip};
    for (int i = 0; i < 6; ++i) {
      if (!p->oW3[i]) continue;
      const W3Shape w = w3_shape(p, i);
      const int j = pa.njobs++;
      pa.W[j] = wsrc[i]; pa.ldw[j] = w.ldw; pa.rows[j] = w.rows; pa.K[j] = w.K; pa.trans[j] = w.trans;
      pa.out[j] = at<unsigned short>(ws, p->oW3[i]);
    }
  }
  if (fused_pro) {
    // status word + flags, weight planes, both chains' images, embedding and D-sep prepend: one launch
    pa.sig = P->sig; pa.gate = P->gate; pa.sig_b = P->sig_b; pa.gate_b = P->gate_b; pa.res = P->res; pa.res_b = P->res_b;
    pa.fout = at<unsigned short>(ws, p->oWPKX); pa.bout = at<float>(ws, p->oWPKB);
    pa.L = L; pa.Cr = Cr; pa.Cd = Cd; pa.skip_b = P->skip_b; pa.Cs = p->Cs; pa.bsum = bsum;
    pa.lc_sig = P->lc_sig; pa.lc_gate = P->lc_gate; pa.Lo = p->Lo;
    pa.lcout = lcx ? at<unsigned short>(ws, p->oLCX) : nullptr; pa.lc16 = p->fwd_nw != 0;
    pa.q = wav_q; pa.pre = P->pre; pa.pre_b = P->pre_b; pa.X = X; pa.xls = p->x_layer_stride; pa.save = save;
    pa.nbl = p->nbl; pa.B = B; pa.T = T; pa.H = H; pa.Q = p->Q;
    pa.zero = at<char>(ws, p->oSTATUS); pa.zero_bytes = 16 + 2 * p->nflag_bytes;
    if ((e = lbwn_step_prologue_launch(pa, st))) return e;
  } else {
    if (x3 && p->chain &&
        (e = lbwn_pack_layers_fb_x3_launch(P->sig, P->gate, P->sig_b, P->gate_b, P->res, P->res_b,
                                           at<unsigned short>(ws, p->oWPKX), at<float>(ws, p->oWPKB), L, Cr, Cd,
                                           P->skip_b, p->Cs, bsum, P->lc_sig, P->lc_gate, p->Lo,
                                           lcx ? at<unsigned short>(ws, p->oLCX) : nullptr, pst, p->fwd_nw != 0)))
      return e;
    if (pa.njobs && (e = lbwn_split_planes_launch(pa.njobs, pa.W, pa.ldw, pa.rows, pa.K, pa.trans, pa.out, pst)))
      return e;
    // one-hot·PRE + PRE_BIAS == row gather (tmodel.py:53-66, :86-102)
    if ((e = lbwn_embed_launch(wav_q, P->pre, P->pre_b, X, B, T, H, Cr, p->Q, st))) return e;
  }
  Cond cd;
  if ((e = cond_forward(p, P, ws, mel, cd, st))) return e;
  // D-separation prepend for every layer (tmodel.py:122-127)
  if (!fused_pro && (e = lbwn_dsep_prepend_launch(X, p->x_layer_stride, save, L, p->nbl, B, T, H, Cr, st))) return e;
  if (p->chain) {
    // all layers in one persistent launch (tmodel.py:313-325)
    lbwn_chain_args c;
    memset(&c, 0, sizeof(c));
    c.X = X; c.xls = p->x_layer_stride; c.Z = Z; c.ldz = ldz; c.wpack = WPK; c.ids = ids;
    c.wpack_x3 = x3 ? at<unsigned short>(ws, p->oWPKX) : nullptr;
    if (x3 && p->oSG) { c.SG = at<float>(ws, p->oSG); c.sgls = m32(M) * 32; }
    p->fwd_x3 = c.SG != nullptr;
    c.gc_tab = cd.gc_tab; c.gc_ld = cd.gc_ld; c.cond = cd.cond; c.ldcond = cd.ldcond;
    if (lcx) {
      c.lcact = at<float>(ws, p->oLCACT[p->nup - 1]); c.lcimg = at<unsigned short>(ws, p->oLCX); c.Lo = p->Lo;
    }
    c.flags = at<unsigned>(ws, p->oFLAGS); c.status = at<unsigned>(ws, p->oSTATUS);
    c.flags_zeroed = 1;   // zeroed with the status word at the step start
    c.xcd = p->chain_xcd;
    if (p->ctrace_blk >= 0) { c.trace = at<long long>(ws, p->oCTRACE); c.trace_blk = p->ctrace_blk; }
    c.B = B; c.T = T; c.H = H; c.L = L; c.nbl = p->nbl; c.Cr = Cr; c.Cd = Cd; c.grid = p->chain_grid;
    if (c.SG && p->fwd_nw) { c.fwd_nw = p->fwd_nw; c.grid = p->fwd_grid; }
    Probe(p, st, "layer_fwd");
    if ((e = lbwn_chain_fwd_launch(c, st))) return e;
    Probe::end(p, st, "layer_fwd");
  } else {
    for (int l = 0; l < L; ++l) {
      lbwn_layer_args a = layer_base(p, P, WPK, ids, l);
      cd.apply(a, l);
      a.x_in = X + l * p->x_layer_stride;
      a.x_out = (l + 1 < L) ? X + (l + 1) * p->x_layer_stride : nullptr;
      a.z = Z + (long)l * Cd;
      a.ldz = ldz;
      Probe(p, st, "layer_fwd", l, l == 0);
      if ((e = lbwn_layer_fwd_launch(a, st))) return e;
      Probe::end(p, st, "layer_fwd", l, l == L - 1);
    }
  }
  // SAVE_l <- last d rows of [SAVE ++ x_l]  (tmodel.py:165)
  if ((e = lbwn_dsep_save_launch(X, p->x_layer_stride, save, L, p->nbl, B, T, H, Cr, st))) return e;
  // mask bits for the backward's dS / dH1 epilogues: both GEMM ends in the x3q<8> form
  // (p->mbits_ok: LBWN_GEMM_MBITS=0 at plan creation forces the f32-mask fallback; a test compares
  // the two bitwise, tests/test_gpu_parity.py::test_mask_bits_equal_f32_masks)
  p->mb_s = p->mbits_ok && lbwn_gemm_x3q8_form((int)M, p->Cs, (int)ldz, 1, w3(p, ws, W3_SKIP_F) != nullptr, 1, 0) &&
            lbwn_gemm_x3q8_form((int)M, p->Cs, p->Cp, 1, w3(p, ws, W3_POST1_B) != nullptr, 1, 0);
  p->mb_r = p->mbits_ok && lbwn_gemm_x3q8_form((int)M, p->Cp, p->Cs, 1, w3(p, ws, W3_POST1_F) != nullptr, 1, 0) &&
            lbwn_gemm_x3q8_form((int)M, p->Cp, p->Q, 1, w3(p, ws, W3_POST2_B) != nullptr, 1, 0);
  // S = Σ_l (z_l·SKIP_l + b) as ONE GEMM over Zcat (tmodel.py:171-184, :316-320)
  if (P->skip_b && !bsum_done && (e = lbwn_sum_bias_launch(P->skip_b, L, p->Cs, bsum, st))) return e;
  {
    lbwn_gemm_args g = gemm0();
    g.A = Z; g.lda = ldz; g.B = P->skip; g.ldb = p->Cs; g.C = S; g.ldc = p->Cs;
    g.M = (int)M; g.N = p->Cs; g.K = (int)ldz; g.bias = P->skip_b ? bsum : nullptr;
    g.b3 = w3(p, ws, W3_SKIP_F);
    g.row_exact = 1;
    if (p->mb_s) g.mbits_out = at<unsigned long long>(ws, p->oMBS);
    Probe(p, st, "skip_fwd");
    if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
    Probe::end(p, st, "skip_fwd");
  }
  // relu(relu(S)·POST1 + b1)  (tmodel.py:194-203)
  lbwn_gemm_args g = gemm0();
  g.A = S; g.lda = p->Cs; g.B = P->post1; g.ldb = p->Cp; g.C = R2; g.ldc = p->Cp;
  g.M = (int)M; g.N = p->Cp; g.K = p->Cs; g.bias = P->post1_b; g.relu_a = 1; g.relu_out = 1;
  g.b3 = w3(p, ws, W3_POST1_F);
  g.row_exact = 1;
  if (p->mb_r) g.mbits_out = at<unsigned long long>(ws, p->oMBR);
  Probe(p, st, "post1_fwd");
  if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
  Probe::end(p, st, "post1_fwd");
  // logits = R2·POST2 + b2  (tmodel.py:204-209)
  g = gemm0();
  g.A = R2; g.lda = p->Cp; g.B = P->post2; g.ldb = p->Q; g.C = LOG; g.ldc = p->Q;
  g.M = (int)M; g.N = p->Q; g.K = p->Cp; g.bias = P->post2_b;
  g.b3 = w3(p, ws, W3_POST2_F);
  g.row_exact = 1;
  Probe(p, st, "post2_fwd");
  if ((e = lbwn_gemm_launch(g, 1, 0, 1, nullptr, st))) return e;
  Probe::end(p, st, "post2_fwd");
  // masked softmax-xent (+ unnormalised dlogits in place)  (tmodel.py:228-249)
  lbwn_head_args h;
  h.logits = LOG; h.q = wav_q; h.ids = ids; h.B = B; h.T = T; h.Q = p->Q;
  h.partial = at<float>(ws, p->oHEADP); h.write_grad = 1;
  // the post2 bias gradient's column partials from the head itself (bf16-split form, Q <= 512),
  // summed in the backward by colsum_final: no colsum pass over dlogits
  h.colpart = (lbwn_gemm_mode() == 1 && p->Q <= 512) ? at<float>(ws, p->oCOLS) : nullptr;
  p->head_colparts = h.colpart ? lbwn_head_nblocks(M, true) : 0;
  int nb = 0;
  Probe(p, st, "head");
  if ((e = lbwn_head_launch(h, &nb, st))) return e;
  Probe::end(p, st, "head");
  return lbwn_stats_reduce_launch(h.partial, nb, stats, st);
}

// Backward (tmodel.py:338-340, TF autodiff of the graph above): head/skip GEMMs, then the
// residual stack in reverse (one persistent chain launch, or one launch per layer), then
// one batched reduction of every layer's weight-gradient partials, then dPRE.
int lbwn_train_backward(lbwn_plan* p, const lbwn_params* P, const lbwn_params* G, void* ws, const int* wav_q,
                        const int* ids, const float* mel, void* stream) {
  LBWN_REQUIRE(p && P && G && ws && wav_q && ids, "train_backward: null argument");
  LBWN_REQUIRE(p->Lo == 0 || mel, "train_backward: LC arch needs the mel input");
  hipStream_t st = (hipStream_t)stream;
  int e;
  if ((e = ensure_device(p))) return e;
  // the backward consumes the forward's layout choices (SG rows, the head's column partials, dZ in
  // chain order), which follow the GEMM arithmetic: a mode switch in between would mix two paths
  LBWN_REQUIRE(p->fwd_mode >= 0, "train_backward: no forward on this plan");
  LBWN_REQUIRE(p->fwd_mode == lbwn_gemm_mode(),
               "train_backward: the GEMM mode changed since the forward (%d -> %d); run the forward again",
               p->fwd_mode, lbwn_gemm_mode());
  // padded head widths: the forward's padded images, gradients into padded buffers
  const lbwn_params* Gref = G;
  lbwn_params Ppad, Gpad;
  if ((e = head_pad_params(p, P, ws, Ppad, false, st))) return e;
  if ((e = head_pad_grads(p, G, ws, Gpad))) return e;
  P = &Ppad;
  G = &Gpad;
  const int L = p->L, B = p->B, T = p->T, Cr = p->Cr, Cd = p->Cd, Cs = p->Cs, Cp = p->Cp, Q = p->Q;
  const long M = p->M, ldz = (long)L * Cd;
  float* X = at<float>(ws, p->oX);
  float* Z = at<float>(ws, p->oZ);
  float* S = at<float>(ws, p->oS);
  float* R2 = at<float>(ws, p->oR2);
  float* LOG = at<float>(ws, p->oLOG);
  float* DH = at<float>(ws, p->oDH);
  float* DS = at<float>(ws, p->oDS);
  float* DZ = at<float>(ws, p->oDZ);
  float* SPL = at<float>(ws, p->oSPLIT);
  float* COLS = at<float>(ws, p->oCOLS);
  lbwn_gemm_args g;
  // dH1 = dlogits·POST2ᵀ ⊙ (R2 > 0)
  g = gemm0();
  g.A = LOG; g.lda = Q; g.B = P->post2; g.ldb = Q; g.C = DH; g.ldc = Cp; g.M = (int)M; g.N = Cp; g.K = Q;
  g.mask = R2; g.ldm = Cp;
  g.b3 = w3(p, ws, W3_POST2_B);
  g.row_exact = 1;
  if (p->mb_r) g.mbits = at<unsigned long long>(ws, p->oMBR);   // (R2 > 0) from post1's epilogue
  // bias-gradient column partials straight from the epilogues (bf16-split form)
  float* CPART = at<float>(ws, p->oCPART);
  const bool fcols = lbwn_gemm_mode() == 1;
  if (fcols && G->post1_b) g.colpart = CPART;
  Probe(p, st, "dh");
  if ((e = lbwn_gemm_launch(g, 1, 1, 1, nullptr, st))) return e;
  Probe::end(p, st, "dh");
  // dS = dH1·POST1ᵀ ⊙ (S > 0)
  g = gemm0();
  g.A = DH; g.lda = Cp; g.B = P->post1; g.ldb = Cp; g.C = DS; g.ldc = Cs; g.M = (int)M; g.N = Cs; g.K = Cp;
  g.mask = S; g.ldm = Cs;
  g.b3 = w3(p, ws, W3_POST1_B);
  g.row_exact = 1;
  if (p->mb_s) g.mbits = at<unsigned long long>(ws, p->oMBS);   // (S > 0) from the skip GEMM's epilogue
  if (fcols && G->skip_b) g.colpart = CPART + (long)lbwn_colpart_parts(M) * Cp;
  Probe(p, st, "ds");
  if ((e = lbwn_gemm_launch(g, 1, 1, 1, nullptr, st))) return e;
  Probe::end(p, st, "ds");
  // dZ = dS·SKIPcatᵀ; for the bf16-split chain in its row-load order (1-KiB runs per load
  // instruction instead of one 16-B piece per row)
  const bool dz_chain = p->chain && p->fwd_x3 && lbwn_gemm_mode() == 1;
  g = gemm0();
  g.A = DS; g.lda = Cs; g.B = P->skip; g.ldb = Cs; g.C = DZ; g.ldc = ldz; g.M = (int)M; g.N = (int)ldz; g.K = Cs;
  g.b3 = w3(p, ws, W3_SKIP_B);
  if (dz_chain) g.c_chain_ls = m32(M) * 32;
  g.xcd2d = p->dz_xcd2d;
  Probe(p, st, "dz");
  if ((e = lbwn_gemm_launch(g, 1, 1, 1, nullptr, st))) return e;
  Probe::end(p, st, "dz");
  // (the final sums on aux2 beside dPOST2 / dPOST1, joined before the chain; LBWN_COLSUM_SIDE=0: in line)
  const bool cs_side = p->colsum_side && p->aux2 && p->chain;
  bool cs_forked = false;
  // bias gradients (column sums of dlogits, dH1, dS; every layer's SKIP_BIAS gets the same Σ dS):
  // here on the main stream, before the fork (small kernels on the least-priority stream beside a
  // resident chain can wait hundreds of µs for a CU)
  {
    const float* cx[3];
    long cld[3];
    int cn[3], cacc[3] = {0, 0, 0}, nj = 0;
    float* cout[3];
    auto job = [&](const float* x, int n, float* o) { cx[nj] = x; cld[nj] = n; cn[nj] = n; cout[nj] = o; ++nj; };
    if (!fcols) {
      if (G->post2_b) job(LOG, Q, G->post2_b);
      if (G->post1_b) job(DH, Cp, G->post1_b);
      if (G->skip_b) job(DS, Cs, G->skip_b);
      if (nj && (e = lbwn_colsum_multi_launch(nj, cx, cld, cn, cout, cacc, (int)M, COLS, st))) return e;
    } else {   // dlogits: first pass here; dH1 / dS partials came from the GEMM epilogues
      float* fp[3];
      float* fo[3];
      int fn[3], fa[3] = {0, 0, 0}, np[3], nf = 0;
      int rp[3] = {1, 1, 1};
      if (G->post2_b) {
        int n0 = p->head_colparts;   // written by this step's head
        if (!n0 && (e = lbwn_colsum_partial_launch(LOG, Q, (int)M, Q, COLS, &n0, st))) return e;
        fp[nf] = COLS; fn[nf] = Q; fo[nf] = G->post2_b; np[nf] = n0; ++nf;
      }
      if (G->post1_b) { fp[nf] = CPART; fn[nf] = Cp; fo[nf] = G->post1_b; np[nf] = lbwn_colpart_parts(M); ++nf; }
      if (G->skip_b) {   // every layer's SKIP_BIAS row gets the same sum: L copies
        fp[nf] = CPART + (long)lbwn_colpart_parts(M) * Cp; fn[nf] = Cs; fo[nf] = G->skip_b;
        np[nf] = lbwn_colpart_parts(M); rp[nf] = L; ++nf;
      }
      hipStream_t cst = st;
      if (nf && cs_side) {
        LBWN_HIP(hipEventRecord(p->ev_cs, st));
        LBWN_HIP(hipStreamWaitEvent(p->aux2, p->ev_cs, 0));
        cst = p->aux2;
      }
      if (nf && (e = lbwn_colsum_final_launch(nf, fp, fn, fo, fa, np, cst, rp))) return e;
      if (nf && cs_side) LBWN_HIP(hipEventRecord(p->ev_cs_done, p->aux2));
      cs_forked = nf && cs_side;
    }
    if (!fcols && G->skip_b && (e = lbwn_bcast_rows_launch(G->skip_b, L, Cs, st))) return e;
  }
  // weight gradients of the head GEMMs (dPOST2, dPOST1) on the main stream BEFORE the chain at
  // full rate: a chain block takes a whole CU's LDS, so nothing runs beside it, and side-stream
  // blocks dispatched before it would hold CUs its lock-step tiles wait for (forked after the
  // chain they shared the chip with dSKIP and ran slower).  dSKIP follows the chain.
  auto dskip = [&](hipStream_t s2, float* spl) -> int {
    int e2;
    lbwn_gemm_args gk = gemm0();
    gk.A = Z; gk.lda = ldz; gk.B = DS; gk.ldb = Cs; gk.C = G->skip; gk.ldc = Cs; gk.M = (int)ldz; gk.N = Cs;
    gk.K = (int)M;
    Probe(p, s2, "dskip");
    if ((e2 = lbwn_gemm_launch(gk, 0, 0, p->split_skip, spl, s2))) return e2;
    Probe::end(p, s2, "dskip");
    return 0;
  };
  auto head_wgrads = [&](hipStream_t ws_st, float* WSPL) -> int {
    int e2;
    // dPOST2 = R2ᵀ·dlogits (db2 = Σ dlogits: the column sums above)
    lbwn_gemm_args gk = gemm0();
    gk.A = R2; gk.lda = Cp; gk.B = LOG; gk.ldb = Q; gk.C = G->post2; gk.ldc = Q; gk.M = Cp; gk.N = Q; gk.K = (int)M;
    Probe(p, ws_st, "dpost2");
    if ((e2 = lbwn_gemm_launch(gk, 0, 0, p->split_post2, WSPL, ws_st))) return e2;
    Probe::end(p, ws_st, "dpost2");
    // dPOST1 = relu(S)ᵀ·dH1
    gk = gemm0();
    gk.A = S; gk.lda = Cs; gk.relu_a = 1; gk.B = DH; gk.ldb = Cp; gk.C = G->post1; gk.ldc = Cp; gk.M = Cs;
    gk.N = Cp; gk.K = (int)M;
    Probe(p, ws_st, "dpost1");
    if ((e2 = lbwn_gemm_launch(gk, 0, 0, p->split_post1, WSPL, ws_st))) return e2;
    Probe::end(p, ws_st, "dpost1");
    return 0;
  };
  if ((e = head_wgrads(st, SPL))) return e;
  if (cs_forked) LBWN_HIP(hipStreamWaitEvent(st, p->ev_cs_done, 0));
  // residual stack in reverse (conditioning recomputed from the forward's GCTAB / COND)
  Cond cd;
  if (p->Ge > 0) {
    cd.gc_tab = at<float>(ws, p->oGCTAB);
    cd.gc_ld = 2L * L * Cd;
    cd.gc_dtab = at<float>(ws, p->oGCD);
    if ((e = lbwn_zero_launch(cd.gc_dtab, sizeof(float) * (size_t)L * p->ncat1 * 2 * Cd, st))) return e;
  }
  if (p->Lo > 0) {
    // the bf16-split backward chain reads no conditioning; the f32 chain and the per-layer
    // kernels recompute the gate from COND, which an in-chain-LC forward did not write
    const bool reads_cond = !(p->chain && p->fwd_x3 && lbwn_gemm_mode() == 1);
    if (reads_cond && !p->cond_valid && (e = cond_project(p, P, ws, st))) return e;
    cd.cond = at<float>(ws, p->oCOND);
    cd.ldcond = 2L * L * Cd;
    cd.dv_out = at<float>(ws, p->oDVALL);
  }
  const float* WPK = at<float>(ws, p->oWPK);
  if (!p->wpk_valid && !(p->chain && p->fwd_x3 && lbwn_gemm_mode() == 1)) {
    // the forward skipped the f32 images (bf16-split chains) but this backward takes an f32 path
    if ((e = lbwn_pack_layers_launch(P->sig, P->gate, P->sig_b, P->gate_b, P->res, P->res_b,
                                     at<float>(ws, p->oWPK), L, Cr, Cd, st)))
      return e;
    p->wpk_valid = true;
  }
  const int sstr = lbwn_layer_slab_stride();
  float* SLABS = at<float>(ws, p->oSLAB);
  if (p->chain) {
    const bool b16 = p->bwd_nw && p->fwd_x3 && lbwn_gemm_mode() == 1;
    const int tpb = lbwn_chain_fwd_tile(b16 ? p->bwd_nw : 0);
    const int ntiles = B * ((T + tpb - 1) / tpb);
    lbwn_chain_args c;
    memset(&c, 0, sizeof(c));
    c.X = X; c.xls = p->x_layer_stride; c.DZ = DZ; c.ldz = ldz; c.wpack = WPK; c.ids = ids;
    if (p->fwd_x3 && lbwn_gemm_mode() == 1) {   // bf16-split backward: no gate recompute (SG)
      c.Z = Z; c.SG = at<float>(ws, p->oSG); c.sgls = m32(M) * 32; c.bimg = at<float>(ws, p->oWPKB);
      c.dzls = m32(M) * 32;   // dZ in chain order (the dZ GEMM above)
      if (cd.gc_dtab) c.tile_gid = at<int>(ws, p->oTGID);
      if (cd.dv_out) c.dvks = m32(M) * 32;   // DV k-blocked: contiguous GEMM k-steps for dlc / dLCcat
    }
    c.slab = SLABS; c.ocg = at<float>(ws, p->oOCG); c.ocls = M * 32;
    c.gc_tab = cd.gc_tab; c.gc_ld = cd.gc_ld; c.cond = cd.cond; c.ldcond = cd.ldcond;
    c.gc_dtab = cd.gc_dtab; c.dv_out = cd.dv_out; c.lddv = cd.ldcond;
    // export form: the weight gradients come from layer_wgrad_kernel below
    const bool wgo = b16 && p->wg_out && p->bwd_nw == 8;
    if (wgo) {
      c.dv_out = at<float>(ws, p->oDVALL); c.lddv = 2L * L * Cd; c.dvks = m32(M) * 32;
      c.gx = at<float>(ws, p->oGX); c.gxls = m32(M) * 32;
      c.tile_gid = nullptr;
    }
    p->dv_blk = c.dvks != 0;
    c.dx0_a = at<float>(ws, p->oGA[0]); c.dx0_c = at<float>(ws, p->oGC0[0]);
    c.flags = at<unsigned>(ws, p->oFLAGS + p->nflag_bytes); c.status = at<unsigned>(ws, p->oSTATUS);
    c.xcd = p->chain_xcd;
    c.flags_zeroed = p->bwd_flags_fresh ? 1 : 0;   // zeroed at the step start unless already used
    p->bwd_flags_fresh = false;
    if (p->ctrace_blk >= 0) { c.trace = at<long long>(ws, p->oCTRACE); c.trace_blk = p->ctrace_blk; }
    c.B = B; c.T = T; c.H = p->H; c.L = L; c.nbl = p->nbl; c.Cr = Cr; c.Cd = Cd; c.grid = p->chain_grid;
    if (b16) { c.bwd_nw = p->bwd_nw; c.grid = p->bwd_grid; }
    Probe(p, st, "layer_bwd");
    if ((e = lbwn_chain_bwd_launch(c, st))) return e;
    Probe::end(p, st, "layer_bwd");
    int wg_parts = ntiles;   // slab partials per layer
    if (wgo) {
      lbwn_wgrad_args wa;
      memset(&wa, 0, sizeof(wa));
      wa.X = X; wa.xls = p->x_layer_stride; wa.Z = Z; wa.lddz = ldz;
      wa.DV = c.dv_out; wa.dvks = c.dvks; wa.GX = c.gx; wa.gxls = c.gxls;
      wa.slab = SLABS; wa.stride = sstr;
      if (cd.gc_dtab) {
        wa.ids = ids; wa.tile_gid = at<int>(ws, p->oTGID); wa.gcs = at<float>(ws, p->oGCS);
        wa.gtab = cd.gc_dtab; wa.gc_ld = cd.gc_ld;
      }
      wa.B = B; wa.T = T; wa.H = p->H; wa.L = L; wa.nbl = p->nbl;
      wa.tpc = lbwn_layer_wgrad_tiles_per_chunk(ntiles, L, p->ncu);
      wg_parts = (ntiles + wa.tpc - 1) / wa.tpc;
      Probe(p, st, "layer_wgrad");
      if ((e = lbwn_layer_wgrad_launch(wa, st))) return e;
      Probe::end(p, st, "layer_wgrad");
    }
    // slab reduction + dPRE on the second side stream (HBM-bound, beside dSKIP's MFMA work)
    hipStream_t rst = st;
    if (p->aux2) {
      rst = p->aux2;
      LBWN_HIP(hipEventRecord(p->ev_chain, st));
      LBWN_HIP(hipStreamWaitEvent(rst, p->ev_chain, 0));
      p->bwd_chain_event = true;
    }
    lbwn_layer_red_args r;
    r.slab = SLABS; r.nparts = wg_parts; r.stride = sstr; r.Cr = Cr; r.Cd = Cd;
    r.dsig = G->sig; r.dgate = G->gate; r.dres = G->res;
    r.dbsig = G->sig_b; r.dbgate = G->gate_b; r.dbres = G->res_b;
    // Side stream (the higher priority), beside the main stream's dlc (LC archs) and dSKIP:
    // dLCcat = lcᵀ·DV first while dlc takes one round of blocks (C5), then dPRE and the slab
    // reduction (the small scatter grid starts while the main stream's GEMM blocks still leave
    // room: step -0.5 %) and the GC table grads.  When dlc needs more than one
    // round of blocks (C4: 512 tiles), dLCcat's higher-priority blocks took its CUs and both
    // streamed the 1.7 GB DV export at once (dlc 1235 us, alone 584): there dLCcat follows the
    // LC upsample backward on the main stream.
    float* SPLA = p->oSPLIT_AUX ? at<float>(ws, p->oSPLIT_AUX) : SPL;
    const bool lc_seq = p->Lo > 0 && (p->M + 255) / 256 * (long)p->split_dlcx > p->ncu;
    if (lc_seq) {   // dlc, the upsample backward and dLCcat first; the side stream then runs beside dSKIP
      if ((e = lc_dlc(p, P, ws, SPL, st))) return e;
      if ((e = lc_upsample_bwd(p, P, G, ws, mel, SPL, st, st))) return e;
      if ((e = lc_wgrad(p, G, ws, SPL, st))) return e;
      if (rst != st) {
        LBWN_HIP(hipEventRecord(p->ev_dlc, st));
        LBWN_HIP(hipStreamWaitEvent(rst, p->ev_dlc, 0));
      }
    }
    if (p->Lo > 0 && !lc_seq && (e = lc_wgrad(p, G, ws, SPLA, rst))) return e;
    if ((e = lbwn_pre_grad_launch(wav_q, at<float>(ws, p->oGA[0]), at<float>(ws, p->oGC0[0]), 1, B, T, Cr, Q, G->pre,
                                  G->pre_b, at<float>(ws, p->oSPLIT2), rst)))
      return e;
    Probe(p, rst, "layer_reduce");
    if ((e = lbwn_layer_reduce_all_launch(r, L, (long)wg_parts * sstr, rst))) return e;
    Probe::end(p, rst, "layer_reduce");
    if (c.tile_gid && (e = lbwn_gc_tile_sum_launch(SLABS, L, ntiles, c.tile_gid, cd.gc_dtab, cd.gc_ld, p->ncat1, rst)))
      return e;
    if (wgo && cd.gc_dtab &&
        (e = lbwn_gc_tile_sum_rows_launch(at<float>(ws, p->oGCS), L, ntiles, at<int>(ws, p->oTGID), cd.gc_dtab,
                                          cd.gc_ld, p->ncat1, rst)))
      return e;
    if ((e = gc_backward(p, P, G, ws, rst))) return e;
    // main stream: dlc, the LC upsample backward (it needs dlc), [dLCcat,] then dSKIP below
    if (p->Lo > 0) {
      if (!lc_seq && (e = lc_dlc(p, P, ws, SPL, st))) return e;
      if (!lc_seq && (e = lc_upsample_bwd(p, P, G, ws, mel, SPL, st, rst))) return e;   // its frame sum on the side
    }
    if (p->aux2) {
      LBWN_HIP(hipEventRecord(p->ev_join2, rst));
      p->bwd_side_event = true;
    }
  } else {
    p->dv_blk = false;
      for (int l = L - 1; l >= 0; --l) {
      lbwn_layer_args a = layer_base(p, P, WPK, ids, l);
      cd.apply(a, l);
      a.x_in = X + l * p->x_layer_stride;
      a.dz_skip = DZ + (long)l * Cd;
      a.lddz = ldz;
      if (l + 1 < L) {
        a.g_a = at<float>(ws, p->oGA[(l + 1) & 1]);
        a.g_c0 = at<float>(ws, p->oGC0[(l + 1) & 1]);
        a.g_d = 1 << ((l + 1) % p->nbl);
      }
      a.out_a = at<float>(ws, p->oGA[l & 1]);
      a.out_c0 = at<float>(ws, p->oGC0[l & 1]);
      a.slab = SLABS + (long)l * p->nblk * sstr;
      a.slab_stride = sstr;
      Probe(p, st, "layer_bwd", l, l == L - 1);
      if ((e = lbwn_layer_bwd_launch(a, st))) return e;
      Probe::end(p, st, "layer_bwd", l, l == 0);
    }
    lbwn_layer_red_args r;
    r.slab = SLABS; r.nparts = p->nblk; r.stride = sstr; r.Cr = Cr; r.Cd = Cd;
    r.dsig = G->sig; r.dgate = G->gate; r.dres = G->res;
    r.dbsig = G->sig_b; r.dbgate = G->gate_b; r.dbres = G->res_b;
    if ((e = lbwn_layer_reduce_all_launch(r, L, (long)p->nblk * sstr, st))) return e;
  }
  if (!p->chain) {
    if ((e = gc_backward(p, P, G, ws, st))) return e;
    if (p->Lo > 0) {
      if ((e = lc_wgrad(p, G, ws, SPL, st))) return e;
      if ((e = lc_dlc(p, P, ws, SPL, st))) return e;
      if ((e = lc_upsample_bwd(p, P, G, ws, mel, SPL, st))) return e;
    }
  }
  if ((e = dskip(st, SPL))) return e;
  // dx_0 = (g + dcur) + shift(dprev) formed inside the scatter; dPRE = onehot(q)ᵀ·dx_0, dPRE_BIAS = Σ dx_0
  // (the chain path enqueued it on the second side stream above)
  if (!p->chain && (e = lbwn_pre_grad_launch(wav_q, at<float>(ws, p->oGA[0]), at<float>(ws, p->oGC0[0]), 1, B, T,
                                             Cr, Q, G->pre, G->pre_b, at<float>(ws, p->oSPLIT2), st)))
    return e;
  if (p->chain && p->aux2) LBWN_HIP(hipStreamWaitEvent(st, p->ev_join2, 0));
  if ((e = head_unpad_grads(p, Gref, ws, st))) return e;
  return 0;
}
