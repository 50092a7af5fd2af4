// extern "C" surface of liblbwn.so (declared in include/lbwn.h).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/lbwn.h"
#include "common.h"
#include "kernels.h"

static thread_local char g_err[1024] = "";

void lbwn_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" {

const char* lbwn_last_error(void) { return g_err; }
int lbwn_abi_version(void) { return LBWN_ABI_VERSION; }

int lbwn_adam_tf1(float* params, const float* grads, float* m, float* v, int64_t n_weights, int64_t n_total,
                  float lr, float beta1, float beta2, float eps, float l2_factor, const float* stats,
                  int64_t* counters, const uint32_t* step_status, void* stream) {
  LBWN_REQUIRE(params && grads && m && v && counters, "adam_tf1: null argument");
  LBWN_REQUIRE(n_weights >= 0 && n_weights <= n_total, "adam_tf1: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  const unsigned* ss = (const unsigned*)step_status;
  int e = lbwn_adam_launch2(params, grads, m, v, (long)n_weights, (long)n_total, lr, beta1, beta2, eps, l2_factor,
                            stats, (const long long*)counters, ss, st);
  if (e) return e;
  if (stats) return lbwn_counters_launch((long long*)counters, stats, 1, ss, st);
  return 0;
}

int lbwn_mulaw_encode(const float* x, int* q, int64_t n, int n_quanta, int tf32, void* stream) {
  LBWN_REQUIRE(n >= 0 && n_quanta >= 2, "mulaw_encode: bad arguments");
  if (n == 0) return 0;
  return lbwn_mulaw_encode_launch(x, q, (long)n, n_quanta, tf32, (hipStream_t)stream);
}

int lbwn_mulaw_decode(const int* q, float* x, int64_t n, int n_quanta, void* stream) {
  LBWN_REQUIRE(n >= 0 && n_quanta >= 2, "mulaw_decode: bad arguments");
  if (n == 0) return 0;
  return lbwn_mulaw_decode_launch(q, x, (long)n, n_quanta, (hipStream_t)stream);
}

int lbwn_gemm_f32(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb, int b_kcontig, float* C,
                  int64_t ldc, int M, int N, int K, const float* bias, int relu_a, int relu_out, const float* mask,
                  int64_t ldm, int accumulate, int split_k, float* slab_ws, void* stream) {
  lbwn_gemm_args g;
  memset(&g, 0, sizeof(g));
  g.A = A; g.lda = (long)lda; g.B = B; g.ldb = (long)ldb; g.C = C; g.ldc = (long)ldc;
  g.M = M; g.N = N; g.K = K; g.bias = bias; g.relu_a = relu_a; g.relu_out = relu_out;
  g.mask = mask; g.ldm = (long)ldm; g.accumulate = accumulate;
  return lbwn_gemm_launch(g, a_kcontig, b_kcontig, split_k, slab_ws, (hipStream_t)stream);
}

int lbwn_gemm_f32_presplit(const float* A, int64_t lda, int a_kcontig, const uint16_t* b3, int N, const float* B,
                           int64_t ldb, int b_kcontig, float* C, int64_t ldc, int M, int K, const float* bias,
                           int relu_a, int relu_out, const float* mask, int64_t ldm, int accumulate, void* stream) {
  LBWN_REQUIRE(b3 != nullptr, "gemm_f32_presplit: b3 is null");
  // the x3r/x3q kernels read b3 with 16-byte loads over lbwn_split_planes_elems(N, K) elements
  LBWN_REQUIRE(((uintptr_t)b3 & 15) == 0, "gemm_f32_presplit: b3 must be 16-byte aligned");
  lbwn_gemm_args g;
  memset(&g, 0, sizeof(g));
  g.A = A; g.lda = (long)lda; g.B = B; g.ldb = (long)ldb; g.C = C; g.ldc = (long)ldc;
  g.M = M; g.N = N; g.K = K; g.bias = bias; g.relu_a = relu_a; g.relu_out = relu_out;
  g.mask = mask; g.ldm = (long)ldm; g.accumulate = accumulate; g.b3 = (const unsigned short*)b3;
  return lbwn_gemm_launch(g, a_kcontig, b_kcontig, 1, nullptr, (hipStream_t)stream);
}

int64_t lbwn_split_planes_elems_abi(int rows, int K) { return (int64_t)lbwn_split_planes_elems(rows, K); }

int lbwn_split_planes(const float* W, int64_t ldw, int rows, int K, int trans, uint16_t* out, void* stream) {
  const long l = (long)ldw;
  unsigned short* o = (unsigned short*)out;
  return lbwn_split_planes_launch(1, &W, &l, &rows, &K, &trans, &o, (hipStream_t)stream);
}

int lbwn_gemm_set_mode(int mode) { return lbwn_gemm_set_mode_impl(mode); }
int lbwn_gemm_get_mode(void) { return lbwn_gemm_mode(); }

int lbwn_layer_image_floats_abi(void) { return lbwn_layer_image_floats(); }

int lbwn_layer_forward(const float* x_in, float* x_out, float* z, int64_t ldz, const float* w_sig,
                       const float* w_gate, const float* b_sig, const float* b_gate, const float* w_res,
                       const float* b_res, const float* gc_tab, const int* ids, const float* cond, int64_t ldcond,
                       int B, int T, int H, int dilation, int n_res, int n_dil, float* wpack_ws, void* stream) {
  LBWN_REQUIRE(x_in && z && w_sig && w_gate && w_res && wpack_ws, "layer_forward: null argument");
  LBWN_REQUIRE(!gc_tab || ids, "layer_forward: gc_tab needs ids");
  lbwn_layer_args a;
  memset(&a, 0, sizeof(a));
  a.x_in = x_in; a.x_out = x_out; a.z = z; a.ldz = (long)ldz;
  a.w_sig = w_sig; a.w_gate = w_gate; a.b_sig = b_sig; a.b_gate = b_gate; a.w_res = w_res; a.b_res = b_res;
  a.gc_tab = gc_tab; a.ids = ids; a.cond = cond; a.ldcond = (long)ldcond;
  a.B = B; a.T = T; a.H = H; a.d = dilation; a.Cr = n_res; a.Cd = n_dil;
  a.wpack = wpack_ws;
  if (int e = lbwn_pack_layers_launch(w_sig, w_gate, b_sig, b_gate, w_res, b_res, wpack_ws, 1, n_res, n_dil,
                                      (hipStream_t)stream))
    return e;
  return lbwn_layer_fwd_launch(a, (hipStream_t)stream);
}

// workspace of lbwn_layer_backward: packed image | per-tile weight-gradient slabs | out_a | out_c0
int64_t lbwn_layer_backward_ws_floats(int B, int T, int n_res) {
  const long M = (long)B * T;
  return (int64_t)lbwn_layer_image_floats() + (int64_t)lbwn_layer_bwd_grid(B, T) * lbwn_layer_slab_stride() +
         2 * (int64_t)M * n_res + 64;
}

int lbwn_layer_backward(const float* x_in, const float* dz, int64_t lddz, const float* dx_out, const float* w_sig,
                        const float* w_gate, const float* b_sig, const float* b_gate, const float* w_res,
                        const float* b_res, const float* gc_tab, const int* ids, const float* cond, int64_t ldcond,
                        float* dx_in, float* dw_sig, float* dw_gate, float* db_sig, float* db_gate, float* dw_res,
                        float* db_res, float* dcond, int64_t lddcond, float* gc_dtab, int B, int T, int H, int dilation,
                        int n_res, int n_dil, float* ws, void* stream) {
  LBWN_REQUIRE(x_in && dz && w_sig && w_gate && w_res && dx_in && dw_sig && dw_gate && dw_res && ws,
               "layer_backward: null argument");
  LBWN_REQUIRE(!gc_tab || ids, "layer_backward: gc_tab needs ids");
  LBWN_REQUIRE(!gc_dtab || gc_tab, "layer_backward: gc_dtab needs gc_tab");
  LBWN_REQUIRE(!dcond || cond, "layer_backward: dcond needs cond");
  LBWN_REQUIRE((((uintptr_t)ws) & 15) == 0, "layer_backward: workspace must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)B * T;
  float* img = ws;
  float* slab = img + lbwn_layer_image_floats();
  const int nblk = lbwn_layer_bwd_grid(B, T), sstr = lbwn_layer_slab_stride();
  float* out_a = slab + (long)nblk * sstr;
  out_a += (16 - ((uintptr_t)out_a & 15)) / 4 % 4;
  float* out_c0 = out_a + M * n_res;
  lbwn_layer_args a;
  memset(&a, 0, sizeof(a));
  a.x_in = x_in; a.dz_skip = dz; a.lddz = (long)lddz;
  a.g_a = dx_out; a.g_c0 = nullptr; a.g_d = 0;   // the caller's dL/dx_{l+1}, already combined
  a.w_sig = w_sig; a.w_gate = w_gate; a.b_sig = b_sig; a.b_gate = b_gate; a.w_res = w_res; a.b_res = b_res;
  a.gc_tab = gc_tab; a.ids = ids; a.cond = cond; a.ldcond = (long)ldcond;
  a.dv_out = dcond; a.lddv = (long)lddcond; a.gc_dtab = gc_dtab;
  a.out_a = out_a; a.out_c0 = out_c0;
  a.slab = slab; a.slab_stride = sstr;
  a.B = B; a.T = T; a.H = H; a.d = dilation; a.Cr = n_res; a.Cd = n_dil;
  a.wpack = img;
  if (int e = lbwn_pack_layers_launch(w_sig, w_gate, b_sig, b_gate, w_res, b_res, img, 1, n_res, n_dil, st)) return e;
  if (int e = lbwn_layer_bwd_launch(a, st)) return e;
  lbwn_layer_red_args r;
  memset(&r, 0, sizeof(r));
  r.slab = slab; r.nparts = nblk; r.stride = sstr; r.Cr = n_res; r.Cd = n_dil;
  r.dsig = dw_sig; r.dgate = dw_gate; r.dres = dw_res; r.dbsig = db_sig; r.dbgate = db_gate; r.dbres = db_res;
  if (int e = lbwn_layer_reduce_launch(r, st)) return e;
  return lbwn_layer_dx_combine_launch(out_a, out_c0, dx_in, B, T, H, dilation, n_res, st);
}

int lbwn_dsep_prepend(float* x_all, int64_t xls, const float* save, int n_layers, int nbl, int B, int T, int H,
                      int n_res, void* stream) {
  LBWN_REQUIRE(H >= (1 << (nbl - 1)), "dsep_prepend: halo %d < max dilation", H);
  return lbwn_dsep_prepend_launch(x_all, (long)xls, save, n_layers, nbl, B, T, H, n_res, (hipStream_t)stream);
}

int lbwn_dsep_save(const float* x_all, int64_t xls, float* save, int n_layers, int nbl, int B, int T, int H,
                   int n_res, void* stream) {
  LBWN_REQUIRE(H >= (1 << (nbl - 1)), "dsep_save: halo %d < max dilation", H);
  return lbwn_dsep_save_launch(x_all, (long)xls, save, n_layers, nbl, B, T, H, n_res, (hipStream_t)stream);
}

int lbwn_head_xent(float* logits, const int* wav_q, const int* ids, int B, int T, int Q, int write_grad, float* stats,
                   float* partial_ws, void* stream) {
  LBWN_REQUIRE(logits && wav_q && ids && stats && partial_ws, "head_xent: null argument");
  LBWN_REQUIRE(T >= 2, "head_xent: slice_sz must be >= 2");
  lbwn_head_args h;
  h.logits = logits; h.q = wav_q; h.ids = ids; h.B = B; h.T = T; h.Q = Q; h.partial = partial_ws;
  h.write_grad = write_grad;
  h.colpart = nullptr;
  int nb = 0;
  hipStream_t st = (hipStream_t)stream;
  if (int e = lbwn_head_launch(h, &nb, st)) return e;
  return lbwn_stats_reduce_launch(partial_ws, nb, stats, st);
}

}  // extern "C"
