// Whole-model engine: the TinyGPT step (model_tiny_gpt.py:297-352 forward, its autograd
// for loss.backward() at loop.py:1233) sequenced natively as stream-ordered kernel
// launches.  The flat parameter layout (one fp32 buffer, grads in the same layout, an
// optional bf16 shadow for the MFMA GEMMs) is owned here; Python builds reference-named
// nn.Parameter views over it (state_dict compatible with the reference).
#include <hip/hip_runtime.h>
#include <string.h>
#include <algorithm>
#include <string>
#include <vector>
#include "../../include/codonlm_hip.h"

extern "C" int cg_rope_tab(int dtype, void* qkv, long long ldqkv, int B, int T, int H, int KV, int hd,
                           const float* cos_tab, const float* sin_tab, int inverse, void* stream);

namespace {

constexpr long long ALIGN = 64;  // elements
inline long long rup(long long a, long long b) { return (a + b - 1) / b * b; }
inline uint32_t site_seed(uint32_t seed, int layer, int site) {
  uint32_t x = seed * 0x01000193u + (uint32_t)layer * 0x9E37u + (uint32_t)site * 0x7F4A7C15u + 0x3C6EF372u;
  x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}
enum { SITE_EMB = 0, SITE_ATTN = 1, SITE_MLP = 2 };

struct Dims {
  int V, Vp, Tmax, L, H, KV, d, hd, kvd, Nqkv, hid, Hp, swiglu, rope;
  int Vh;  // split-bf16 dlogits half width: Vp rounded to 32, so the head dX product's K = 2 Vh is a
           // multiple of the persistent tile's 64-deep k-step
  int G, dw_bm, dw_ks;  // blocks per grouped weight-gradient launch, its tile rows, token split
  int force_ks;         // cfg.opts.dw_ksplit: 0 = the planner's choice
  bool rem_first;       // cfg.opts.dw_remainder_first
  long long plan_tokens;  // cfg.opts.dw_plan_tokens: plan as for this many tokens (0 = the step's)
};

bool dims_of(const cg_model_cfg* c, Dims& D) {
  if (!c || c->n_embd <= 0 || c->n_head <= 0 || c->n_embd % c->n_head) return false;
  // engine options (zero = defaults): out-of-range values are an error, not a silent default
  if (c->opts.dw_group < 0 || c->opts.dw_ksplit < 0 || c->opts.dw_ksplit > 3 || c->opts.dw_plan_tokens < 0 ||
      c->opts.attn_bwd_algo < CG_ATTN_BWD_AUTO || c->opts.attn_bwd_algo > CG_ATTN_BWD_FUSED ||
      c->opts.pers_max_wg < 0 || c->opts.attn_mask_kernel < 0 || c->opts.attn_mask_kernel > 2)
    return false;
  D.V = c->vocab_size;
  D.Vp = (int)rup(c->vocab_size, 16);
  D.Vh = (int)rup(D.Vp, 32);
  D.Tmax = c->block_size;
  D.L = c->n_layer;
  D.H = c->n_head;
  D.KV = (c->n_kv_head > 0 && c->n_kv_head <= c->n_head) ? c->n_kv_head : c->n_head;
  D.d = c->n_embd;
  D.hd = c->n_embd / c->n_head;
  D.kvd = D.KV * D.hd;
  D.Nqkv = D.d + 2 * D.kvd;
  D.swiglu = c->use_swiglu != 0;
  D.rope = c->use_rope != 0;
  D.hid = D.swiglu ? (int)(8 * (long long)c->n_embd / 3) : 4 * c->n_embd;
  D.Hp = D.swiglu ? (int)rup(D.hid, 64) : D.hid;
  D.G = 1;
  D.dw_bm = 128;
  D.dw_ks = 1;
  D.force_ks = c->opts.dw_ksplit;
  D.rem_first = c->opts.dw_remainder_first != 0;
  D.plan_tokens = c->opts.dw_plan_tokens;
  return true;
}

// Group size and tiles of the grouped dW launches (bf16 engine).  A group's tiles run as one
// persistent launch with one workgroup per CU and every tile costing about the same (full-token
// reduction), so a group takes ceil(tiles / CUs) rounds of its tile's cost.  Tile candidates
// (cg_gemm_dw_tiles codes): 128 x 128 (cost 1), 256 x 128 (1.38: twice the work in 1.38x the
// time) and 256 x 256 (2.35: 4x the work; a 2-stage ring, its DMA latency partly exposed),
// measured at K = 16384 on the C4/C5 shapes (tools/dw_grouped.py).  Each group takes its
// cheapest tile (a short remainder group often prefers the smaller tile); the plan minimises the
// summed cost of the groups (G, G, ..., remainder) and, on ties, prefers the smaller group (its
// gradients are final -- and all-reduced -- earlier).  cg_model_cfg.opts.dw_group / dw_ksplit force
// a choice (tests, A/B runs).
struct DwPlan {
  int G, bm, ks;  // group size, tile of a full group, its token-range split
};
// weight elements of one block's dW products (the slab a token-range split writes per slice)
static long long dw_block_elems(const Dims& D) {
  const long long d = D.d;
  return (long long)D.Nqkv * d + d * d + (D.swiglu ? 3LL * D.Hp * d : 2LL * D.hid * d);
}
// cheapest (tile, token-range split) for a group of n blocks over M tokens, and its cost.  A split
// into ks slices makes ks x more work items of 1/ks the k-steps (more rounds filled where the
// tiles alone leave CUs idle: C2's 144 tiles on 256 CUs) plus a slab pass of ~20 B per weight
// element and extra slice at ~5 TB/s, priced against ~11 ns per token for 1.0 of tile cost
// (C2 / C3 rocprofv3: 495 us for a round of 1.38 at M = 32768)
static int dw_tile_for(const Dims& D, int n, double* cost_out, int* ks_out, long long M) {
  if (D.plan_tokens > 0) M = D.plan_tokens;
  const int d = D.d, cus = cg_pers_cus();
  int best = 256, best_ks = 1;
  double best_cost = 1e30;
  for (int bm : {128, 256, 512}) {
    // (256 x 256: 2.35 at K = 16384 on C4/C5; 2.49 at C3, K = 32768: 951 vs 526 us per round of
    // the 256 x 128 tile, rocprofv3 -- 2.5 keeps C4 on its 5/5/2 plan and moves C3 from 6/4 to
    // 4/4/2, 9.08 -> 8.99 ms/step, profiles/round4/dw_sweep)
    const double tile_cost = bm == 128 ? 1.0 : bm == 256 ? 1.38 : 2.5;
    const int per_layer = cg_gemm_dw_tiles(bm, D.Nqkv, d) + cg_gemm_dw_tiles(bm, d, d) +
                          (D.swiglu ? cg_gemm_dw_tiles(bm, 2 * D.Hp, d) + cg_gemm_dw_tiles(bm, d, D.Hp)
                                    : cg_gemm_dw_tiles(bm, D.hid, d) + cg_gemm_dw_tiles(bm, d, D.hid));
    for (int ks = 1; ks <= 3; ++ks) {
      if (D.force_ks && ks != D.force_ks) continue;
      const double slab = (double)(ks - 1) * n * dw_block_elems(D) * 20.0 / 5e12 / (11e-9 * (double)M);
      // the 256 x 128 tile split in two token ranges over several rounds runs 1.35x slower per
      // item than the model's k-loop share: C4 at B = 32, a 4-block group's 768 items took 1003 us
      // against the modelled 796; pricing it so moves that plan from 8/4 to 5/5/2, 14.81 -> 14.64
      // ms/step, with C2 / C3 / C5 on their unchanged plans (profiles/round5/dw_plan_b32.txt)
      const int rounds = (n * per_layer * ks + cus - 1) / cus;
      const double split_pen = (bm == 256 && ks == 2 && rounds >= 2) ? 1.35 : 1.0;
      const double cost = (double)rounds * tile_cost / ks * split_pen + slab;
      if (cost < best_cost - 1e-9) best_cost = cost, best = bm, best_ks = ks;
    }
  }
  if (cost_out) *cost_out = best_cost;
  if (ks_out) *ks_out = best_ks;
  return best;
}
DwPlan dw_plan(const cg_model_cfg* c, const Dims& D, long long M) {
  if (c->dtype != CG_BF16 || D.L <= 0) return {1, 128, 1};
  const int forced_g = c->opts.dw_group;
  const int gmax = std::min(D.L, CG_DW_MAX / 4);
  DwPlan best{1, 128, 1};
  double best_cost = 1e30;
  for (int g = 1; g <= gmax; ++g) {
    if (forced_g && g != std::min(forced_g, gmax)) continue;
    double cost = 0;
    for (int left = D.L; left > 0; left -= g) {
      double cg;
      dw_tile_for(D, std::min(g, left), &cg, nullptr, M);
      cost += cg;
    }
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      int ks = 1;
      const int bm = dw_tile_for(D, g, nullptr, &ks, M);
      best = {g, bm, ks};
    }
  }
  return best;
}

struct Layout {
  std::vector<cg_param_entry> e;
  long long total = 0;
  // per-layer offsets
  struct Lay {
    long long ln1w, ln1b, wqkv, bqkv, wp, bp, ln2w, ln2b, w1, b1, w2, b2, wgu, wd;
  };
  std::vector<Lay> lay;
  long long tok, pos = -1, lnfw, lnfb, head = -1, termw = -1, termb = -1;
  std::vector<long long> off1w, off1b, off2w, off2b;
};

void build_layout(const cg_model_cfg* c, const Dims& D, Layout& Lo) {
  long long cur = 0;
  auto add = [&](int kind, int layer, int rows, int cols, long long ld, long long alloc_elems, bool align) {
    if (align) cur = rup(cur, ALIGN);
    cg_param_entry en{kind, layer, cur, rows, cols, ld};
    Lo.e.push_back(en);
    long long off = cur;
    cur += alloc_elems;
    return off;
  };
  const int d = D.d;
  Lo.tok = add(CG_P_TOK_EMB, -1, D.V, d, d, (long long)D.Vp * d, true);
  if (!D.rope) Lo.pos = add(CG_P_POS_EMB, -1, D.Tmax, d, d, (long long)D.Tmax * d, true);
  Lo.lay.resize(D.L);
  for (int l = 0; l < D.L; ++l) {
    auto& y = Lo.lay[l];
    y.ln1w = add(CG_P_LN1_W, l, d, 0, d, d, true);
    y.ln1b = add(CG_P_LN1_B, l, d, 0, d, d, false);
    y.wqkv = add(CG_P_Q_W, l, d, d, d, (long long)d * d, true);
    add(CG_P_K_W, l, D.kvd, d, d, (long long)D.kvd * d, false);
    add(CG_P_V_W, l, D.kvd, d, d, (long long)D.kvd * d, false);
    y.bqkv = add(CG_P_Q_B, l, d, 0, d, d, true);
    add(CG_P_K_B, l, D.kvd, 0, D.kvd, D.kvd, false);
    add(CG_P_V_B, l, D.kvd, 0, D.kvd, D.kvd, false);
    y.wp = add(CG_P_PROJ_W, l, d, d, d, (long long)d * d, true);
    y.bp = add(CG_P_PROJ_B, l, d, 0, d, d, true);
    y.ln2w = add(CG_P_LN2_W, l, d, 0, d, d, true);
    y.ln2b = add(CG_P_LN2_B, l, d, 0, d, d, false);
    if (!D.swiglu) {
      y.w1 = add(CG_P_FC1_W, l, D.hid, d, d, (long long)D.hid * d, true);
      y.b1 = add(CG_P_FC1_B, l, D.hid, 0, D.hid, D.hid, true);
      y.w2 = add(CG_P_FC2_W, l, d, D.hid, D.hid, (long long)d * D.hid, true);
      y.b2 = add(CG_P_FC2_B, l, d, 0, d, d, true);
      y.wgu = y.wd = -1;
    } else {
      y.wgu = add(CG_P_GATE_W, l, D.hid, d, d, (long long)D.Hp * d, true);
      add(CG_P_UP_W, l, D.hid, d, d, (long long)D.Hp * d, false);
      y.wd = add(CG_P_DOWN_W, l, d, D.hid, D.Hp, (long long)d * D.Hp, true);
      y.w1 = y.b1 = y.w2 = y.b2 = -1;
    }
  }
  Lo.lnfw = add(CG_P_LNF_W, -1, d, 0, d, d, true);
  Lo.lnfb = add(CG_P_LNF_B, -1, d, 0, d, d, false);
  if (!c->tie_embeddings) Lo.head = add(CG_P_HEAD_W, -1, D.V, d, d, (long long)D.Vp * d, true);
  if (c->termination_aux) {
    const int nc = c->termination_n_classes;
    // rows padded to 16 (zero) so the backward products see an extent the bf16 tiles take
    Lo.termw = add(CG_P_TERM_W, -1, nc, d, d, rup(nc, 16) * d, true);
    Lo.termb = add(CG_P_TERM_B, -1, nc, 0, nc, nc, true);
  }
  for (int i = 0; i < c->n_offsets && i < 8; ++i) {
    Lo.off1w.push_back(add(CG_P_OFF1_W, i, d, d, d, (long long)d * d, true));
    Lo.off1b.push_back(add(CG_P_OFF1_B, i, d, 0, d, d, true));
    Lo.off2w.push_back(add(CG_P_OFF2_W, i, d, d, d, (long long)d * d, true));
    Lo.off2b.push_back(add(CG_P_OFF2_B, i, d, 0, d, d, true));
  }
  Lo.total = rup(cur, ALIGN);
}

// ---------------------------------------------------------------------------
// workspace carving
// ---------------------------------------------------------------------------
struct WS {
  char* base = nullptr;
  size_t off = 0;
  template <typename P>
  P* take(size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    P* p = base ? (P*)(base + off) : nullptr;
    off += bytes;
    return p;
  }
};

struct LayerAct {
  float *mean1, *rstd1, *mean2, *rstd2, *lse, *xmid;
  void *h1, *qkv, *y, *h2, *a, *g, *gu, *s;
  // bf16 mode: per-step transposed copies of the shadow weights (K-contiguous dX operands)
  void *qkvT, *pT, *w1T, *w2T, *wguT, *wdT;
  // bf16 training with dropout: this block's attention keep bits (cg_attn_drop_mask), made by
  // the forward and read again by the backward
  void* dmask;
};
// per-block gradient operands kept until the block's grouped dW launch (slot = position of
// the block inside its group): dY of fc2/down (gin), of fc1/gate|up (dmlp), of proj (gattn),
// of qkv (dqkv), all in the compute dtype
struct DwSlot {
  void *gin, *gattn, *dmlp, *dqkv;
  // partial rows of the block's parameter / bias gradient column sums, reduced in one batched
  // launch per dW group (cg_reduce_columns): LayerNorm 2 / 1 backward ([nblk][3d]: dgamma |
  // dbeta | consumer bias), fc1 bias ([ceil(M/64)][hid]), qkv bias ([B*ceil(T/128)][Nqkv])
  float *lnp2, *lnp1, *cpart, *bpart;
};
// byte sizes of the carved scratch buffers handed to the op entry points (their ws_bytes)
struct WsBytes {
  size_t lnp, cpart, colws, splitws, embws, cews, delta, ocp_half, dwslab;
};
struct Acts {
  int32_t* seg;
  std::vector<DwSlot> slot;
  float* x;  // (L+1) x M x d
  std::vector<LayerAct> la;
  float *meanf, *rstdf, *logits_int, *logits_pad;
  void* xf;
  // backward scratch
  void *dlogits, *dbig, *dsmall;
  void* head2;  // bf16 mode: [E^T 0 | E^T 0] (d x 2Vh, K-contiguous), B operand of the split-dlogits dX
  long long ldl;  // dlogits row stride: Vp, or 2 Vh for split bf16 (hi in [0, Vh) | lo in [Vh, 2Vh))
  float *g, *dtmp, *delta, *lnpart, *colws, *splitws, *embws, *cews;
  float* bpart;  // qkv bias-gradient partials from the attention backward [B*ceil(T/128)][Nqkv]
  float* dwslab;  // bf16: the grouped dW's token-split slabs (null when no group splits)
  size_t splitws_floats;
  WsBytes nb;
  bool wT;  // transposed weight copies present
  // auxiliary offset heads: pre-GELU a, GELU output g, projection pj (compute dtype, M x d)
  std::vector<void*> oa, og, opj;
  // their backward dY operands, kept per head until one grouped dW launch takes all of them
  std::vector<void*> odpj, oda;
  // their two d x d weights transposed (wT mode): K-contiguous dX operands, as the blocks'
  std::vector<void*> o1T, o2T;
  // per offset head: its logits gradient (the layout of dlogits), stacked [head][M] like opj, so
  // the tied head's weight gradient over all heads is ONE product reduced over heads x tokens
  std::vector<void*> odl;
  std::vector<float*> ocp;  // their bias-gradient column-sum partials (2 per head), reduced batched
};

constexpr int MAX_SPLIT = 16;

size_t carve(const cg_model_cfg* c, const Dims& D, int B, int T, char* base, Acts& A) {
  WS w{base, 0};
  const long long M = (long long)B * T;
  const size_t es = c->dtype == CG_BF16 ? 2 : 4;
  const int d = D.d;
  A.seg = w.take<int32_t>(M * 4);
  A.x = w.take<float>((size_t)(D.L + 1) * M * d * 4);
  A.la.resize(D.L);
  for (int l = 0; l < D.L; ++l) {
    auto& a = A.la[l];
    a.mean1 = w.take<float>(M * 4); a.rstd1 = w.take<float>(M * 4);
    a.mean2 = w.take<float>(M * 4); a.rstd2 = w.take<float>(M * 4);
    a.lse = w.take<float>((size_t)B * D.H * T * 4);
    a.xmid = w.take<float>(M * d * 4);
    a.h1 = w.take<char>(M * d * es);
    a.qkv = w.take<char>(M * D.Nqkv * es);
    a.y = w.take<char>(M * d * es);
    a.h2 = w.take<char>(M * d * es);
    if (!D.swiglu) {
      a.a = w.take<char>(M * D.hid * es);
      a.g = w.take<char>(M * D.hid * es);
      a.gu = a.s = nullptr;
    } else {
      a.gu = w.take<char>(M * 2 * (size_t)D.Hp * es);
      a.s = w.take<char>(M * (size_t)D.Hp * es);
      a.a = a.g = nullptr;
    }
  }
  A.meanf = w.take<float>(M * 4);
  A.rstdf = w.take<float>(M * 4);
  A.xf = w.take<char>(M * d * es);
  A.logits_int = w.take<float>(M * D.V * 4);
  A.logits_pad = w.take<float>(M * D.Vp * 4);  // head product at N = Vp (vector-epilogue tiles)
  const int noff = std::min(c->n_offsets, 8);
  A.oa.assign(noff, nullptr); A.og.assign(noff, nullptr); A.opj.assign(noff, nullptr);
  A.odpj.assign(noff, nullptr); A.oda.assign(noff, nullptr); A.odl.assign(noff, nullptr);
  A.ocp.assign(noff, nullptr);
  const size_t es_dl = c->dtype == CG_BF16 ? 2 : 4;
  const long long ldl_ = c->dtype == CG_BF16 ? 2LL * D.Vh : D.Vp;
  char* opj_all = noff ? w.take<char>((size_t)noff * M * d * es) : nullptr;
  char* odl_all = noff ? w.take<char>((size_t)noff * M * ldl_ * es_dl) : nullptr;
  A.nb.ocp_half = cg_colsum_workspace((int)M, d);
  for (int i = 0; i < noff; ++i) {
    A.ocp[i] = w.take<float>(2 * A.nb.ocp_half);
    A.opj[i] = opj_all + (size_t)i * M * d * es;
    A.odl[i] = odl_all + (size_t)i * M * ldl_ * es_dl;
    A.odpj[i] = w.take<char>(M * d * es);
    A.oda[i] = w.take<char>(M * d * es);
    A.oa[i] = w.take<char>(M * d * es);
    A.og[i] = w.take<char>(M * d * es);
  }
  A.ldl = ldl_;
  A.dlogits = w.take<char>(M * A.ldl * es);
  A.slot.resize(D.G);
  A.nb.lnp = cg_layernorm_bwd_workspace((int)M, d, 1);
  A.nb.cpart = (size_t)((M + 63) / 64) * std::max(D.hid, d) * 4;
  for (auto& sl : A.slot) {
    sl.gin = w.take<char>(M * d * es);
    sl.gattn = w.take<char>(M * d * es);
    sl.dmlp = w.take<char>(M * (D.swiglu ? 2LL * D.Hp : (long long)D.hid) * es);
    sl.dqkv = w.take<char>(M * D.Nqkv * es);
    sl.lnp2 = w.take<float>(A.nb.lnp);
    sl.lnp1 = w.take<float>(A.nb.lnp);
    sl.cpart = w.take<float>(A.nb.cpart);
    sl.bpart = w.take<float>((size_t)B * ((T + 127) / 128) * D.Nqkv * 4);
  }
  A.head2 = c->dtype == CG_BF16 ? w.take<char>((size_t)2 * D.Vh * d * 2) : nullptr;
  const long long big = std::max<long long>({(long long)D.hid, 2LL * D.Hp, (long long)D.Nqkv});
  A.dbig = w.take<char>(M * big * es);
  A.dsmall = w.take<char>(M * std::max(d, D.Hp) * es);
  A.g = w.take<float>(M * d * 4);
  A.dtmp = w.take<float>(M * d * 4);
  A.nb.delta = cg_attn_bwd_workspace(B, T, D.H);
  A.delta = w.take<float>(A.nb.delta);
  A.lnpart = w.take<float>(A.nb.lnp);
  const long long maxcols = std::max<long long>({big, (long long)d, (long long)D.Hp});
  A.nb.colws = cg_colsum_workspace((int)M, (int)maxcols);
  A.colws = w.take<float>(A.nb.colws);
  A.bpart = w.take<float>((size_t)B * ((T + 127) / 128) * D.Nqkv * 4);
  long long wmax = std::max<long long>({(long long)D.Nqkv * d, (long long)D.hid * d, 2LL * D.Hp * d,
                                        (long long)D.Vp * d, (long long)d * d});
  A.splitws_floats = (size_t)MAX_SPLIT * wmax;
  // also holds the fused bias-gradient column-sum partials ([ceil(M/64)][cols])
  A.splitws_floats = std::max<size_t>(A.splitws_floats, (size_t)((M + 63) / 64) * (size_t)big);
  A.nb.splitws = A.splitws_floats * 4;
  A.splitws = w.take<float>(A.nb.splitws);
  // grouped-dW token-split slabs: (ks - 1) slices of a group's weights (+ the tied head's, which
  // can join the first group), for the larger of the full group's and the remainder's split
  A.dwslab = nullptr;
  A.nb.dwslab = 0;
  if (c->dtype == CG_BF16 && D.L > 0) {
    const int rem = D.L % D.G;
    int ks_rem = 1;
    if (rem) dw_tile_for(D, rem, nullptr, &ks_rem, M);
    const long long head = (long long)D.Vp * d;
    const long long need = std::max<long long>((long long)(D.dw_ks - 1) * (D.G * dw_block_elems(D) + head),
                                               (long long)(ks_rem - 1) * (rem * dw_block_elems(D) + head));
    if (need > 0) {
      A.nb.dwslab = (size_t)need * 4;
      A.dwslab = w.take<float>(A.nb.dwslab);
    }
  }
  A.nb.embws = cg_embed_bwd_workspace((int)B, (int)T, D.V, d);  // bytes, sized by the kernel's own chunking
  A.embws = w.take<float>(A.nb.embws);
  A.nb.cews = cg_ce_workspace((int)M);
  A.cews = w.take<float>(A.nb.cews);
  A.wT = c->dtype == CG_BF16 && d % 8 == 0 && D.Nqkv % 8 == 0 && D.hid % 8 == 0 && D.Hp % 8 == 0;
  for (int l = 0; l < D.L; ++l) {
    auto& a = A.la[l];
    a.qkvT = a.pT = a.w1T = a.w2T = a.wguT = a.wdT = nullptr;
    if (!A.wT) continue;
    a.qkvT = w.take<char>((size_t)d * D.Nqkv * 2);
    a.pT = w.take<char>((size_t)d * d * 2);
    if (!D.swiglu) {
      a.w1T = w.take<char>((size_t)d * D.hid * 2);
      a.w2T = w.take<char>((size_t)D.hid * d * 2);
    } else {
      a.wguT = w.take<char>((size_t)d * 2 * D.Hp * 2);
      a.wdT = w.take<char>((size_t)D.Hp * d * 2);
    }
  }
  const int noffT = A.wT ? std::min(c->n_offsets, 8) : 0;
  A.o1T.assign(noffT, nullptr);
  A.o2T.assign(noffT, nullptr);
  for (int i = 0; i < noffT; ++i) {
    A.o1T[i] = w.take<char>((size_t)d * d * 2);
    A.o2T[i] = w.take<char>((size_t)d * d * 2);
  }
  const bool dmask = c->dtype == CG_BF16 && c->dropout > 0.f;
  for (int l = 0; l < D.L; ++l)
    A.la[l].dmask = dmask ? w.take<char>(cg_attn_drop_mask_bytes(B, T, D.H)) : nullptr;
  return w.off + 256;
}

struct Ctx {
  const cg_model* m;
  Dims D;
  Layout Lo;
  Acts A;
  int B, T;
  long long M;
  int dt;
  hipStream_t s;
};

int make_ctx(const cg_model* m, int B, int T, void* stream, Ctx& C) {
  if (!dims_of(&m->cfg, C.D)) return CG_EINVAL;
  const DwPlan pl = dw_plan(&m->cfg, C.D, (long long)B * T);
  C.D.G = pl.G;
  C.D.dw_bm = pl.bm;
  C.D.dw_ks = pl.ks;
  build_layout(&m->cfg, C.D, C.Lo);
  C.m = m;
  C.B = B; C.T = T; C.M = (long long)B * T;
  C.dt = m->cfg.dtype;
  C.s = (hipStream_t)stream;
  size_t need = carve(&m->cfg, C.D, B, T, nullptr, C.A);
  if (!m->workspace || m->workspace_bytes < need) return CG_EINVAL;
  carve(&m->cfg, C.D, B, T, (char*)m->workspace, C.A);
  return CG_OK;
}

inline const void* W(const Ctx& C, long long off) {
  if (C.dt == CG_BF16) return (const void*)(C.m->shadow + off);
  return (const void*)(C.m->params + off);
}
inline float* P(const Ctx& C, long long off) { return C.m->params + off; }
inline float* G(const Ctx& C, long long off) { return C.m->grads + off; }
inline size_t es(const Ctx& C) { return C.dt == CG_BF16 ? 2 : 4; }
inline void* at(void* p, long long elems, const Ctx& C) { return (char*)p + elems * es(C); }

#define CK(x)                      \
  do {                             \
    int _r = (x);                  \
    if (_r != CG_OK) return _r;    \
  } while (0)

cg_gemm_desc gdesc(const Ctx& C) {
  cg_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.in_dtype = C.dt;
  g.c_dtype = C.dt;
  g.alpha = 1.0f;
  g.split_k = 1;
  g.max_wg = C.m->cfg.opts.pers_max_wg;
  return g;
}

// y[M,N] = x[M,K] . W[N,K]^T  (forward nn.Linear)
cg_gemm_desc lin_fwd(const Ctx& C, const void* x, long long ldx, long long woff, long long ldw, int N, int K, void* y,
                     long long ldy) {
  cg_gemm_desc g = gdesc(C);
  g.M = (int)C.M; g.N = N; g.K = K;
  g.A = x; g.lda = ldx; g.a_kcontig = 1;
  g.B = W(C, woff); g.ldb = ldw; g.b_kcontig = 1;
  g.C = y; g.ldc = ldy;
  return g;
}
// dx[M,K] = dy[M,N] . W[N,K]   (wT: optional [K][N] copy of W -> K-contiguous operand)
cg_gemm_desc lin_dx(const Ctx& C, const void* dy, long long lddy, long long woff, long long ldw, int N, int K, void* dx,
                    long long lddx, const void* wT = nullptr) {
  cg_gemm_desc g = gdesc(C);
  g.M = (int)C.M; g.N = K; g.K = N;
  g.A = dy; g.lda = lddy; g.a_kcontig = 1;
  if (wT) {
    g.B = wT; g.ldb = N; g.b_kcontig = 1;
  } else {
    g.B = W(C, woff); g.ldb = ldw; g.b_kcontig = 0;
  }
  g.C = dx; g.ldc = lddx;
  return g;
}
// d[M,d] (fp32, + resid epilogue set by the caller) = dl[M,Vp] . E[Vp,d] for a head weight E:
// in bf16 mode dl holds split-bf16 rows (hi | lo, CG_BF16X2, halves Vh wide with zero pads) and the
// product runs over K = 2 Vh against [E^T 0 | E^T 0] (A.head2, filled by fill_head2): both operands
// K-contiguous and K a multiple of 64, so it runs on the persistent tile (round 6; it was the
// register-staged vector kernel with an MN-contiguous [E; E], 27.6 us at C4)
cg_gemm_desc head_dx(const Ctx& C, long long hoff, void* out, long long ldo, const void* dl = nullptr) {
  const Dims& D = C.D;
  if (!dl) dl = C.A.dlogits;
  if (C.dt != CG_BF16) return lin_dx(C, dl, D.Vp, hoff, D.d, D.Vp, D.d, out, ldo);
  cg_gemm_desc g = gdesc(C);
  g.M = (int)C.M; g.N = D.d; g.K = 2 * D.Vh;
  g.A = dl; g.lda = C.A.ldl; g.a_kcontig = 1;
  g.B = C.A.head2; g.ldb = 2 * D.Vh; g.b_kcontig = 1;
  g.C = out; g.ldc = ldo;
  return g;
}
int fill_head2(const Ctx& C, long long hoff) {
  if (C.dt != CG_BF16) return CG_OK;
  const Dims& D = C.D;
  // zero pad columns [Vp, Vh) of each half (the matching dlogits pads are zero too), then E^T twice
  if (hipMemsetAsync(C.A.head2, 0, (size_t)2 * D.Vh * D.d * 2, C.s) != hipSuccess) return CG_ELAUNCH;
  cg_transpose_batch tb;
  tb.n = 2;
  for (int i = 0; i < 2; ++i)
    tb.items[i] = cg_transpose_item{W(C, hoff), (char*)C.A.head2 + (size_t)i * D.Vh * 2, D.d, 2LL * D.Vh, D.Vp, D.d};
  return cg_transpose16_batch(&tb, C.s);
}
// refresh the transposed weight copies of every block (one batched launch per 64 matrices)
int transpose_weights(const Ctx& C) {
  if (!C.A.wT) return CG_OK;
  const Dims& D = C.D;
  const int d = D.d;
  cg_transpose_batch tb;
  tb.n = 0;
  auto add = [&](long long off, long long ld, int rows, int cols, void* dst) -> int {
    if (tb.n == CG_TRANSPOSE_MAX) {
      CK(cg_transpose16_batch(&tb, C.s));
      tb.n = 0;
    }
    tb.items[tb.n++] = cg_transpose_item{W(C, off), dst, ld, rows, rows, cols};
    return CG_OK;
  };
  for (int l = 0; l < D.L; ++l) {
    const auto& o = C.Lo.lay[l];
    const auto& a = C.A.la[l];
    CK(add(o.wqkv, d, D.Nqkv, d, a.qkvT));
    CK(add(o.wp, d, d, d, a.pT));
    if (!D.swiglu) {
      CK(add(o.w1, d, D.hid, d, a.w1T));
      CK(add(o.w2, D.hid, d, D.hid, a.w2T));
    } else {
      CK(add(o.wgu, d, 2 * D.Hp, d, a.wguT));
      CK(add(o.wd, D.Hp, d, D.Hp, a.wdT));
    }
  }
  for (size_t i = 0; i < C.A.o1T.size(); ++i) {
    CK(add(C.Lo.off1w[i], d, d, d, C.A.o1T[i]));
    CK(add(C.Lo.off2w[i], d, d, d, C.A.o2T[i]));
  }
  return cg_transpose16_batch(&tb, C.s);
}
int pick_split(const Ctx& C, int Mo, int N, long long K) {
  const int bm = 128;  // the 128x128 tiles of the bf16 and (round 4: every layout) fp32 dW products
  const long long tiles = (long long)((Mo + bm - 1) / bm) * ((N + bm - 1) / bm);
  long long s = (512 + tiles - 1) / tiles;
  long long smax = K / 512;
  if (s > smax) s = smax;
  // 8 slabs suffice once there are >= 32 tiles; the 16-tile products (d x d at d512: attention
  // proj) run 218 -> 291 TF/s with 16 (dw_sweep on the box)
  if (s > (tiles > 16 ? 8 : MAX_SPLIT)) s = tiles > 16 ? 8 : MAX_SPLIT;
  // > 32 tiles with long slabs: the most slabs that still fit one round at 2 blocks per CU
  // (qkv at d512, 48 tiles, K = 16384: 10 slabs 51.6 us vs 8 slabs 55.5 us, dw_sweep on the box)
  if (tiles > 32 && 512 / tiles > s && K / (512 / tiles) >= 1536) s = std::min<long long>(512 / tiles, MAX_SPLIT);
  if (s < 1) s = 1;
  if ((size_t)s * Mo * N > C.A.splitws_floats) s = 1;
  return (int)s;
}
// dW[N,K] (+)= dy[M,N]^T . x[M,K]
int lin_dw(const Ctx& C, const void* dy, long long lddy, const void* x, long long ldx, int N, int K, long long goff,
           long long ldg, int accumulate) {
  cg_gemm_desc g = gdesc(C);
  g.c_dtype = CG_F32;
  g.M = N; g.N = K; g.K = (int)C.M;
  g.A = dy; g.lda = lddy; g.a_kcontig = 0;
  g.B = x; g.ldb = ldx; g.b_kcontig = 0;
  g.C = G(C, goff); g.ldc = ldg;
  g.epilogue = accumulate ? CG_EPI_ACCUM : 0;
  g.split_k = pick_split(C, N, K, C.M);
  g.workspace = C.A.splitws;
  g.ws_bytes = C.A.nb.splitws;
  return cg_gemm(&g, C.s);
}
int bias_grad(const Ctx& C, const void* dy, long long lddy, int N, long long goff, int accumulate) {
  return cg_colsum(C.dt, dy, lddy, (int)C.M, N, G(C, goff), accumulate, C.A.colws, C.A.nb.colws, C.s);
}

float train_p(const cg_model* m) { return m->training ? m->cfg.dropout : 0.0f; }

// dW groups run from block L-1 downwards.  Order 1 (default since round 4): the short remainder
// group (L mod G blocks) comes LAST (C4: groups of 5, 5, 2 from the top), so the buckets whose
// all-reduce can only start after the final dW launch are the short group's (25 MB instead of
// 63 MB at C4).  Order 0 (cg_model_opts.dw_remainder_first): the remainder first (2, 5, 5), so the first buckets
// are final after 2 blocks instead of 5.  tools/bucket_replay.py priced both on one GPU with the
// all-reduces modelled as CU-holding side-stream kernels: 5/5/2 8.22 / 8.44 ms against 2/5/5
// 8.31 / 8.63 ms per C4 step at 600 / 300 GB/s bus bandwidth.
int first_group(const Dims& D) { return (D.rem_first && D.L % D.G) ? D.L % D.G : D.G; }
// position of block l inside its group, counted from the group's top block
int slot_of(const Dims& D, int l) {
  const int u = D.L - 1 - l, f = first_group(D);
  return u < f ? u : (u - f) % D.G;
}
bool group_ends(const Dims& D, int l) {
  if (l == 0) return true;
  const int u = D.L - 1 - l, f = first_group(D);
  return u < f ? u == f - 1 : slot_of(D, l) == D.G - 1;
}

// Parameter / bias gradient reductions deferred to the end of a dW group: the LayerNorm
// backward and the fused column-sum epilogues of a group's blocks leave partial rows in their
// slots; one cg_reduce_columns launch per group turns them into gradients (per-layer reduce
// launches were ~5 us each, mostly idle GPU).  The batch lives in the model (its lifetime and
// thread ownership follow the model's); phase 0 starts a backward.
cg_reduce_batch& pending(const cg_model* m) { return const_cast<cg_model*>(m)->reduce_pending; }
int defer_reduce(const cg_model* m, const float* part, long long ld, int nrows, int cols, float* dst, int accumulate,
                 void* stream) {
  cg_reduce_batch& b = pending(m);
  if (b.n == CG_REDUCE_MAX) {  // full (only with very small groups of very many jobs): drain
    CK(cg_reduce_columns(&b, stream));
    b.n = 0;
  }
  cg_reduce_job& j = b.j[b.n++];
  j.part = part; j.ld = ld; j.nrows = nrows; j.cols = cols; j.dst = dst; j.accumulate = accumulate;
  j.first_block = 0;
  return CG_OK;
}
int flush_reduce(const cg_model* m, void* stream) {
  cg_reduce_batch& b = pending(m);
  const int rc = b.n ? cg_reduce_columns(&b, stream) : CG_OK;
  b.n = 0;
  return rc;
}
// LayerNorm backward whose dgamma / dbeta (/ consumer bias) reductions join the pending batch
int ln_bwd_deferred(const Ctx& C, int dy_dtype, const void* dy, const float* x, const float* mean, const float* rstd,
                    long long gw, const float* g_in, void* g_out_t, uint32_t seed, float p, float* part, float* dgamma,
                    float* dbeta, float* dcol, int accumulate) {
  const int d = C.D.d;
  CK(cg_layernorm_bwd_partials(dy_dtype, dy, d, x, d, mean, rstd, P(C, gw), g_in, C.A.g, C.dt, g_out_t, seed, p, part,
                               C.A.nb.lnp, dcol ? 1 : 0, (int)C.M, d, C.s));
  const int nw = dcol ? 3 : 2;
  const int nblk = cg_layernorm_bwd_blocks((int)C.M);
  CK(defer_reduce(C.m, part, (long long)nw * d, nblk, d, dgamma, accumulate, C.s));
  CK(defer_reduce(C.m, part + d, (long long)nw * d, nblk, d, dbeta, accumulate, C.s));
  if (dcol) CK(defer_reduce(C.m, part + 2 * d, (long long)nw * d, nblk, d, dcol, accumulate, C.s));
  return CG_OK;
}

// column sums of dy [M][d] (a bias gradient) as partial rows joining the pending batch
int defer_colsum(const Ctx& C, const void* dy, float* part, long long goff, int accumulate) {
  int np = 0;
  CK(cg_colsum_partials(C.dt, dy, C.D.d, (int)C.M, C.D.d, part, C.A.nb.ocp_half, &np, C.s));
  return defer_reduce(C.m, part, C.D.d, np, C.D.d, G(C, goff), accumulate, C.s);
}

// d(head weight) (+)= alpha dlogits^T . xf  (M_out = Vp: pad rows of dlogits are zero; the hi
// half of split-bf16 rows) as a split-K product of its own
int head_dw_now(const Ctx& C, long long hoff, float alpha, int accumulate) {
  const Acts& A = C.A;
  cg_gemm_desc g = gdesc(C);
  g.c_dtype = CG_F32;
  g.M = C.D.Vp; g.N = C.D.d; g.K = (int)C.M;
  g.A = A.dlogits; g.lda = A.ldl; g.a_kcontig = 0;
  g.B = A.xf; g.ldb = C.D.d; g.b_kcontig = 0;
  g.C = G(C, hoff); g.ldc = C.D.d;
  g.epilogue = accumulate ? CG_EPI_ACCUM : 0;
  g.alpha = alpha;
  g.split_k = pick_split(C, C.D.Vp, C.D.d, C.M);
  g.workspace = A.splitws;
  g.ws_bytes = A.nb.splitws;
  return cg_gemm(&g, C.s);
}
// The tied head's weight gradient, deferred from phase 0 into the first dW group's grouped
// launch (bf16, no aux heads): a few more tiles beside the group's (the C4 remainder group fills
// 192 of 256 CUs) instead of a split-K product (22 us) and its slab reduction (7 us).  Its
// operands (dlogits, xf) are not written again before that launch, and the tied gradient
// (tok_emb) is final only after phase 2, so no data-parallel bucket sees it early.  The pending
// product lives in the cg_model itself (head_dw_*), so its lifetime and thread ownership are the
// model's; phase 0 (re)sets it, phase 2 runs it if no group did.
}  // namespace

namespace {

// The tile code and the token split the grouped dW launch of blocks [l_lo, l_hi] runs with (the
// split only where the slab workspace exists)
int group_plan(const Ctx& C, int l_hi, int l_lo, int* ks_out) {
  const Dims& D = C.D;
  int ks = D.dw_ks;
  const int tile = l_hi - l_lo + 1 == D.G ? D.dw_bm : dw_tile_for(D, l_hi - l_lo + 1, nullptr, &ks, C.M);
  *ks_out = (ks > 1 && C.A.dwslab) ? ks : 1;
  return tile;
}
// fc1's bias gradient (the column sums of dH) comes from block l's grouped dW launch when that
// launch does not split the tokens (gemm_dw.h CS variant); else from the dGELU product's epilogue
bool fc1_bias_in_dw(const Ctx& C, int l) {
  const Dims& D = C.D;
  if (C.dt != CG_BF16 || D.swiglu) return false;
  const int top = l + slot_of(D, l);
  int lo = top;
  while (!group_ends(D, lo)) --lo;
  int ks = 1;
  group_plan(C, top, lo, &ks);
  return ks == 1;
}

// The weight gradients of blocks [l_lo, l_hi] from their kept operands: one grouped launch in
// bf16 mode (gemm_dw.h), the per-product GEMMs in fp32 parity mode.
int flush_dw(const Ctx& C, int l_hi, int l_lo, int accumulate) {
  const Dims& D = C.D;
  const int d = D.d;
  cg_dw_group grp;
  memset(&grp, 0, sizeof(grp));
  grp.max_wg = C.m->cfg.opts.pers_max_wg;
  grp.K = (int)C.M;
  int ks = 1;
  grp.tile_m = group_plan(C, l_hi, l_lo, &ks);
  if (ks > 1) {
    grp.ksplit = ks;
    grp.workspace = C.A.dwslab;
    grp.ws_bytes = C.A.nb.dwslab;
  }
  auto add = [&](const void* dy, int n_out, const void* x, int k_out, long long goff) -> int {
    if (C.dt != CG_BF16) return lin_dw(C, dy, n_out, x, k_out, n_out, k_out, goff, k_out, accumulate);
    cg_dw_product& q = grp.p[grp.n++];
    q.A = dy; q.lda = n_out;
    q.B = x; q.ldb = k_out;
    q.C = G(C, goff); q.ldc = k_out;
    q.N_out = n_out; q.K_out = k_out;
    q.alpha = 1.0f; q.accumulate = accumulate;
    return CG_OK;
  };
  for (int l = l_hi; l >= l_lo; --l) {
    const auto& o = C.Lo.lay[l];
    const auto& a = C.A.la[l];
    const DwSlot& sl = C.A.slot[slot_of(D, l)];
    if (!D.swiglu) {
      CK(add(sl.gin, d, a.g, D.hid, o.w2));
      CK(add(sl.dmlp, D.hid, a.h2, d, o.w1));
      if (C.dt == CG_BF16 && ks == 1) grp.p[grp.n - 1].col_sum = G(C, o.b1);  // fc1_bias_in_dw
    } else {
      CK(add(sl.gin, d, a.s, D.Hp, o.wd));
      CK(add(sl.dmlp, 2 * D.Hp, a.h2, d, o.wgu));
    }
    CK(add(sl.gattn, d, a.y, d, o.wp));
    CK(add(sl.dqkv, D.Nqkv, a.h1, d, o.wqkv));
  }
  cg_model* mm = const_cast<cg_model*>(C.m);
  if (mm->head_dw_pending && C.dt == CG_BF16 && grp.n < CG_DW_MAX) {
    cg_dw_product& q = grp.p[grp.n++];
    q.A = C.A.dlogits; q.lda = C.A.ldl;
    q.B = C.A.xf; q.ldb = d;
    q.C = G(C, mm->head_dw_off); q.ldc = d;
    q.N_out = D.Vp; q.K_out = d;
    q.alpha = mm->head_dw_alpha; q.accumulate = mm->head_dw_accumulate;
    mm->head_dw_pending = 0;
  }
  if (C.dt == CG_BF16 && grp.n) return cg_gemm_dw_grouped(&grp, C.s);
  return CG_OK;
}

int zero_grad(const Ctx& C, long long off, long long elems) {
  return hipMemsetAsync(G(C, off), 0, (size_t)elems * 4, C.s) == hipSuccess ? CG_OK : CG_ELAUNCH;
}

// Backward of the auxiliary heads (model_tiny_gpt.py:329-337) inside phase 0: parameter grads
// of termination_head / offset_projs, the tied head's extra gradient, and their share of dxf
// (added into A.dtmp before the ln_f backward).  A.dlogits is free here (head products done).
int aux_backward(const Ctx& C, int accumulate) {
  const cg_model* m = C.m;
  const Dims& D = C.D;
  const Acts& A = C.A;
  const int d = D.d;
  const long long M = C.M;
  const long long hoff = m->cfg.tie_embeddings ? C.Lo.tok : C.Lo.head;
  // the offset heads' two d x d weight gradients each -- and the termination head's -- (bf16: one
  // grouped launch after the loop, as the blocks' dW; their dY operands stay in per-head buffers)
  cg_dw_group grp;
  memset(&grp, 0, sizeof(grp));
  grp.max_wg = C.m->cfg.opts.pers_max_wg;
  grp.K = (int)M;
  grp.tile_m = 128;  // 10 products of d x d at C5: the 128-row tile gives the most workgroups
  if (m->cfg.termination_aux) {
    const int nc = m->cfg.termination_n_classes, ncp = (int)rup(nc, 16);
    if (m->d_term_logits) {
      if (!m->aux_ready || m->ld_d_term < nc) return CG_EINVAL;
      CK(cg_cast_pad_2d(m->d_term_logits, m->ld_d_term, (int)M, nc, C.dt, A.dlogits, ncp, ncp, C.s));
      // dW_t = dT^T . xf over the padded rows (pad rows of dT^T are zero): bf16 in the grouped launch
      // (A.dlogits is not written again before it), fp32 as its own split-K product
      if (C.dt == CG_BF16) {
        cg_dw_product& q = grp.p[grp.n++];
        q.A = A.dlogits; q.lda = ncp;
        q.B = A.xf; q.ldb = d;
        q.C = G(C, C.Lo.termw); q.ldc = d;
        q.N_out = ncp; q.K_out = d;
        q.alpha = 1.0f; q.accumulate = accumulate;
      } else {
        cg_gemm_desc g = gdesc(C);
        g.c_dtype = CG_F32;
        g.M = ncp; g.N = d; g.K = (int)M;
        g.A = A.dlogits; g.lda = ncp; g.a_kcontig = 0;
        g.B = A.xf; g.ldb = d; g.b_kcontig = 0;
        g.C = G(C, C.Lo.termw); g.ldc = d;
        g.epilogue = accumulate ? CG_EPI_ACCUM : 0;
        g.split_k = pick_split(C, ncp, d, M);
        g.workspace = A.splitws;
        g.ws_bytes = A.nb.splitws;
        CK(cg_gemm(&g, C.s));
      }
      CK(cg_colsum(CG_F32, m->d_term_logits, m->ld_d_term, (int)M, nc, G(C, C.Lo.termb), accumulate, A.colws,
                   A.nb.colws, C.s));
      cg_gemm_desc g = gdesc(C);
      // dxf += dT . W_t
      g = lin_dx(C, A.dlogits, ncp, C.Lo.termw, d, ncp, d, A.dtmp, d);
      g.c_dtype = CG_F32;
      g.epilogue = CG_EPI_RESID; g.resid = A.dtmp; g.ldr = d;
      CK(cg_gemm(&g, C.s));
    } else if (!accumulate) {
      CK(zero_grad(C, C.Lo.termw, (long long)ncp * d));
      CK(zero_grad(C, C.Lo.termb, nc));
    }
  }
  const int noff = std::min(m->cfg.n_offsets, 8);
  auto add_dw = [&](const void* dy, const void* x, long long goff) -> int {
    if (C.dt != CG_BF16) return lin_dw(C, dy, d, x, d, d, d, goff, d, accumulate);
    cg_dw_product& q = grp.p[grp.n++];
    q.A = dy; q.lda = d;
    q.B = x; q.ldb = d;
    q.C = G(C, goff); q.ldc = d;
    q.N_out = d; q.K_out = d;
    q.alpha = 1.0f; q.accumulate = accumulate;
    return CG_OK;
  };
  for (int i = 0; i < noff; ++i) {
    const float* dl = m->d_offset_logits[i];
    if (!dl) {
      if (!accumulate) {
        CK(zero_grad(C, C.Lo.off1w[i], (long long)d * d));
        CK(zero_grad(C, C.Lo.off1b[i], d));
        CK(zero_grad(C, C.Lo.off2w[i], (long long)d * d));
        CK(zero_grad(C, C.Lo.off2b[i], d));
      }
      continue;
    }
    if (!m->aux_ready) return CG_EINVAL;
    CK(cg_cast_pad_2d(dl, D.V, (int)M, D.V, C.dt == CG_BF16 ? CG_BF16X2 : C.dt, A.odl[i], A.ldl,
                      C.dt == CG_BF16 ? D.Vh : D.Vp, C.s));
    // dpj = Gc . E ; the second Linear's grads
    void* dpj = A.odpj[i];
    void* da = A.oda[i];
    cg_gemm_desc g = head_dx(C, hoff, dpj, d, A.odl[i]);
    g.c_dtype = C.dt;
    CK(cg_gemm(&g, C.s));
    CK(add_dw(dpj, A.og[i], C.Lo.off2w[i]));
    CK(defer_colsum(C, dpj, A.ocp[i], C.Lo.off2b[i], accumulate));
    // da = (dpj . W2) * gelu'(a) ; the first Linear's grads
    const bool hasT = i < (int)A.o2T.size();
    g = lin_dx(C, dpj, d, C.Lo.off2w[i], d, d, d, da, d, hasT ? A.o2T[i] : nullptr);
    g.epilogue = CG_EPI_DGELU | CG_EPI_GELU_DERIV; g.aux = A.oa[i]; g.ld_aux = d;
    CK(cg_gemm(&g, C.s));
    CK(add_dw(da, A.xf, C.Lo.off1w[i]));
    CK(defer_colsum(C, da, A.ocp[i] + cg_colsum_workspace((int)M, d) / 4, C.Lo.off1b[i], accumulate));
    // dxf += da . W1
    g = lin_dx(C, da, d, C.Lo.off1w[i], d, d, d, A.dtmp, d, hasT ? A.o1T[i] : nullptr);
    g.c_dtype = CG_F32;
    g.epilogue = CG_EPI_RESID; g.resid = A.dtmp; g.ldr = d;
    CK(cg_gemm(&g, C.s));
  }
  // d(head) += sum_i Gc_i^T . pj_i over the heads with a gradient: one product reduced over
  // (head, token) rows -- the logits gradients and pj operands are stacked per head (phase 0's own
  // head product initialised it; hi half of split rows)
  for (int first = 0; first < noff;) {  // one product per run of consecutive heads with a gradient
    if (!m->d_offset_logits[first]) {
      ++first;
      continue;
    }
    int cnt = 1;
    while (first + cnt < noff && m->d_offset_logits[first + cnt]) ++cnt;
    cg_gemm_desc g = gdesc(C);
    g.c_dtype = CG_F32;
    g.M = D.Vp; g.N = d; g.K = (int)(M * cnt);
    g.A = A.odl[first]; g.lda = A.ldl; g.a_kcontig = 0;
    g.B = A.opj[first]; g.ldb = d; g.b_kcontig = 0;
    g.C = G(C, hoff); g.ldc = d;
    g.epilogue = CG_EPI_ACCUM;
    // a few output tiles over a long reduction: more slabs than pick_split's cap (16) so the
    // launch fills the chip (~1 k-row per slab), bounded by the slab workspace
    long long sk = std::max<long long>(pick_split(C, D.Vp, d, M * cnt), std::min<long long>(96, M * cnt / 1024));
    while (sk > 1 && (size_t)sk * D.Vp * d > A.splitws_floats) --sk;
    g.split_k = (int)sk;
    g.workspace = A.splitws;
    g.ws_bytes = A.nb.splitws;
    CK(cg_gemm(&g, C.s));
    first += cnt;
  }
  if (grp.n) {
    int rc = cg_gemm_dw_grouped(&grp, C.s);
    for (int j = 0; rc == CG_EUNSUPPORTED && j < grp.n; ++j) {  // unaligned shapes: per product
      const cg_dw_product& q = grp.p[j];
      const int r2 = lin_dw(C, q.A, q.lda, q.B, q.ldb, q.N_out, q.K_out, q.C - m->grads, q.ldc, accumulate);
      if (r2 != CG_OK) return r2;
      if (j == grp.n - 1) rc = CG_OK;
    }
    CK(rc);
  }
  return CG_OK;
}

}  // namespace

// ===========================================================================
extern "C" int cg_model_param_layout(const cg_model_cfg* cfg, cg_param_entry* out, int max, long long* total) {
  Dims D;
  if (!dims_of(cfg, D)) return CG_EINVAL;
  Layout Lo;
  build_layout(cfg, D, Lo);
  if (total) *total = Lo.total;
  const int n = (int)Lo.e.size();
  if (out)
    for (int i = 0; i < n && i < max; ++i) out[i] = Lo.e[i];
  return n;
}

extern "C" int cg_model_dw_plan(const cg_model_cfg* cfg, int B, int T, int* group_layers, int* tile_m, int* ksplit) {
  Dims D;
  if (!dims_of(cfg, D) || B <= 0 || T <= 0) return CG_EINVAL;
  const DwPlan pl = dw_plan(cfg, D, (long long)B * T);
  if (group_layers) *group_layers = pl.G;
  if (tile_m) *tile_m = pl.bm;
  if (ksplit) *ksplit = pl.ks;
  return CG_OK;
}

extern "C" size_t cg_model_workspace_bytes(const cg_model_cfg* cfg, int B, int T) {
  Dims D;
  if (!dims_of(cfg, D)) return 0;
  const DwPlan pl = dw_plan(cfg, D, (long long)B * T);
  D.G = pl.G;
  D.dw_bm = pl.bm;
  D.dw_ks = pl.ks;
  Acts A;
  return carve(cfg, D, B, T, nullptr, A);
}

extern "C" int cg_model_forward(cg_model* m, const int64_t* idx, const int64_t* targets, int B, int T, int training,
                                uint32_t seed, int window, float* logits, float* loss, void* stream) {
  if (!m || !idx || B <= 0 || T <= 0) return CG_EINVAL;
  if (T > m->cfg.block_size) return CG_EINVAL;
  if (m->cfg.dtype == CG_BF16 && !m->shadow) return CG_EINVAL;
  if (m->cfg.use_rope && (!m->rope_cos || !m->rope_sin)) return CG_EINVAL;
  m->B = B; m->T = T; m->training = training; m->seed = seed; m->window = window;
  m->idx = idx; m->targets = targets;
  m->aux_ready = 0; m->head_grad_scale = 1.0f; m->head_grad_scale_dev = nullptr;
  m->d_term_logits = nullptr; m->ld_d_term = 0;
  for (int i = 0; i < 8; ++i) m->d_offset_logits[i] = nullptr;
  Ctx C;
  CK(make_ctx(m, B, T, stream, C));
  const Dims& D = C.D;
  const Acts& A = C.A;
  const int d = D.d;
  const long long M = C.M;
  const float p = train_p(m);
  const float eps = m->cfg.ln_eps > 0 ? m->cfg.ln_eps : 1e-5f;
  m->logits = logits ? logits : A.logits_int;

  // the attention keep bits: written by each block's attention forward itself (default), or by the
  // mask kernel right before it (cfg.opts.attn_mask_kernel; a mask pass on a side stream ahead of
  // the forward measured slower, round 2)
  const bool fused_keep = !m->cfg.opts.attn_mask_kernel;
  // attn_mask_kernel 2: the keep words made in the launch of the block's LN1 (cg_layernorm_fwd_mask),
  // read by the forward (round 6)
  const bool mask_in_ln = m->cfg.opts.attn_mask_kernel == 2;
  const bool rope_epi = !m->cfg.opts.rope_tables;
  CK(cg_segment_starts(idx, A.seg, B, T, m->cfg.sep_id, C.s));
  CK(cg_embed_fwd(idx, P(C, C.Lo.tok), C.Lo.pos >= 0 ? P(C, C.Lo.pos) : nullptr, A.x, B, T, d,
                  site_seed(seed, -1, SITE_EMB), p, C.s));
  for (int l = 0; l < D.L; ++l) {
    const auto& o = C.Lo.lay[l];
    const auto& a = A.la[l];
    float* xl = A.x + (size_t)l * M * d;
    float* xn = A.x + (size_t)(l + 1) * M * d;
    const void* dmask = p > 0.f ? a.dmask : nullptr;
    if (dmask && mask_in_ln)  // this block's attention keep words beside its LN1 rows (one launch)
      CK(cg_layernorm_fwd_mask(C.dt, xl, d, P(C, o.ln1w), P(C, o.ln1b), a.h1, d, a.mean1, a.rstd1, (int)M, d, eps, B, T,
                               D.H, site_seed(seed, l, SITE_ATTN), p, a.dmask, C.s));
    else
      CK(cg_layernorm_fwd(C.dt, xl, d, P(C, o.ln1w), P(C, o.ln1b), a.h1, d, a.mean1, a.rstd1, (int)M, d, eps, C.s));
    cg_gemm_desc g = lin_fwd(C, a.h1, d, o.wqkv, d, D.Nqkv, d, a.qkv, D.Nqkv);
    g.epilogue = CG_EPI_BIAS; g.bias = P(C, o.bqkv);
    // RoPE in the projection's epilogue where the GEMM tile implements it, else a table pass
    int rc_rope = CG_EUNSUPPORTED;
    if (D.rope && rope_epi) {
      cg_gemm_desc gr = g;
      gr.epilogue |= CG_EPI_ROPE;
      gr.rope_cos = m->rope_cos; gr.rope_sin = m->rope_sin;
      gr.rope_T = T; gr.rope_hd = D.hd; gr.rope_heads = D.H + D.KV;
      rc_rope = cg_gemm(&gr, C.s);
      if (rc_rope != CG_OK && rc_rope != CG_EUNSUPPORTED) return rc_rope;
    }
    if (rc_rope != CG_OK) {
      CK(cg_gemm(&g, C.s));
      if (D.rope) CK(cg_rope_tab(C.dt, a.qkv, D.Nqkv, B, T, D.H, D.KV, D.hd, m->rope_cos, m->rope_sin, 0, C.s));
    }
    if (dmask && fused_keep) {
      CK(cg_attn_fwd_keep(C.dt, a.qkv, D.Nqkv, m->cfg.sep_id >= 0 ? A.seg : nullptr, a.y, d, a.lse, B, T, D.H, D.KV,
                          D.hd, window, site_seed(seed, l, SITE_ATTN), p, a.dmask, C.s));
    } else {
      if (dmask && !mask_in_ln) CK(cg_attn_drop_mask(B, T, D.H, site_seed(seed, l, SITE_ATTN), p, a.dmask, C.s));
      CK(cg_attn_fwd(C.dt, a.qkv, D.Nqkv, m->cfg.sep_id >= 0 ? A.seg : nullptr, a.y, d, a.lse, B, T, D.H, D.KV, D.hd,
                     window, site_seed(seed, l, SITE_ATTN), p, dmask, C.s));
    }
    g = lin_fwd(C, a.y, d, o.wp, d, d, d, a.xmid, d);
    g.c_dtype = CG_F32;
    g.epilogue = CG_EPI_BIAS | CG_EPI_RESID; g.bias = P(C, o.bp); g.resid = xl; g.ldr = d;
    CK(cg_gemm(&g, C.s));
    CK(cg_layernorm_fwd(C.dt, a.xmid, d, P(C, o.ln2w), P(C, o.ln2b), a.h2, d, a.mean2, a.rstd2, (int)M, d, eps, C.s));
    if (!D.swiglu) {
      g = lin_fwd(C, a.h2, d, o.w1, d, D.hid, d, a.g, D.hid);
      g.epilogue = CG_EPI_BIAS | CG_EPI_GELU | CG_EPI_GELU_DERIV; g.bias = P(C, o.b1); g.aux_out = a.a; g.ld_aux = D.hid;
      CK(cg_gemm(&g, C.s));
      g = lin_fwd(C, a.g, D.hid, o.w2, D.hid, d, D.hid, xn, d);
      g.c_dtype = CG_F32;
      g.epilogue = CG_EPI_BIAS | CG_EPI_RESID | (p > 0 ? CG_EPI_DROPOUT : 0);
      g.bias = P(C, o.b2); g.resid = a.xmid; g.ldr = d;
      g.drop_seed = site_seed(seed, l, SITE_MLP); g.drop_p = p;
      CK(cg_gemm(&g, C.s));
    } else {
      // gate|up product with SwiGLU in its epilogue (s to a.s, pre-activations to a.gu); the
      // separate pass where the fused tile does not apply (fp32, unaligned shapes)
      g = lin_fwd(C, a.h2, d, o.wgu, d, D.Hp, d, a.s, D.Hp);
      g.epilogue = CG_EPI_SWIGLU; g.aux_out = a.gu; g.ld_aux = 2 * D.Hp; g.n_valid = D.hid;
      int rc = C.dt == CG_BF16 ? cg_gemm(&g, C.s) : CG_EUNSUPPORTED;
      if (rc == CG_EUNSUPPORTED) {
        g = lin_fwd(C, a.h2, d, o.wgu, d, 2 * D.Hp, d, a.gu, 2 * D.Hp);
        CK(cg_gemm(&g, C.s));
        rc = cg_swiglu_fwd(C.dt, a.gu, 2 * D.Hp, D.Hp, a.s, D.Hp, (int)M, D.hid, C.s);
      }
      CK(rc);
      g = lin_fwd(C, a.s, D.Hp, o.wd, D.Hp, d, D.Hp, xn, d);
      g.c_dtype = CG_F32;
      g.epilogue = CG_EPI_RESID | (p > 0 ? CG_EPI_DROPOUT : 0);
      g.resid = a.xmid; g.ldr = d;
      g.drop_seed = site_seed(seed, l, SITE_MLP); g.drop_p = p;
      CK(cg_gemm(&g, C.s));
    }
  }
  float* xL = A.x + (size_t)D.L * M * d;
  CK(cg_layernorm_fwd(C.dt, xL, d, P(C, C.Lo.lnfw), P(C, C.Lo.lnfb), A.xf, d, A.meanf, A.rstdf, (int)M, d, eps, C.s));
  const long long hoff = m->cfg.tie_embeddings ? C.Lo.tok : C.Lo.head;
  // the head product runs at N = Vp (zero weight rows V..Vp-1) so that it takes the vector
  // epilogue tiles; the loss reads the padded logits and the caller's (M, V) copy is compacted
  cg_gemm_desc g = lin_fwd(C, A.xf, d, hoff, d, D.Vp, d, A.logits_pad, D.Vp);
  g.c_dtype = CG_F32;
  CK(cg_gemm(&g, C.s));
  CK(cg_cast_pad_2d(A.logits_pad, D.Vp, (int)M, D.V, CG_F32, m->logits, D.V, D.V, C.s));
  if (targets) {
    CK(cg_cross_entropy(A.logits_pad, D.Vp, targets, (int)M, D.V, m->cfg.label_smoothing, m->loss_weights, 0, 1.0f,
                        C.dt == CG_BF16 ? CG_BF16X2 : C.dt, A.dlogits, A.ldl, loss, A.cews, A.nb.cews, C.s));
  }
  return CG_OK;
}

extern "C" int cg_model_aux_forward(cg_model* m, float* term_logits, long long ld_term, float* const* offset_logits,
                                    long long ld_off, void* stream) {
  if (!m || !m->idx || m->B <= 0 || m->T <= 0) return CG_EINVAL;
  const int nc = m->cfg.termination_aux ? m->cfg.termination_n_classes : 0;
  const int noff = std::min(m->cfg.n_offsets, 8);
  if (nc > 0 && (!term_logits || ld_term < nc)) return CG_EINVAL;
  if (noff > 0 && (!offset_logits || ld_off < m->cfg.vocab_size)) return CG_EINVAL;
  for (int i = 0; i < noff; ++i)
    if (!offset_logits[i]) return CG_EINVAL;
  Ctx C;
  CK(make_ctx(m, m->B, m->T, stream, C));
  const Dims& D = C.D;
  const Acts& A = C.A;
  const int d = D.d;
  if (nc > 0) {
    // N padded to the weight's 16 zero-padded rows (an extent the MFMA tiles take; the bias reads of
    // the pad columns stay inside the bias's 256-B aligned slot), then the nc columns copied out.
    // A.dtmp is backward scratch, free until the backward's head products
    const int ncp = (int)rup(nc, 16);
    cg_gemm_desc g = lin_fwd(C, A.xf, d, C.Lo.termw, d, ncp, d, A.dtmp, ncp);
    g.c_dtype = CG_F32;
    g.epilogue = CG_EPI_BIAS; g.bias = P(C, C.Lo.termb);
    CK(cg_gemm(&g, C.s));
    CK(cg_cast_pad_2d(A.dtmp, ncp, (int)C.M, nc, CG_F32, term_logits, ld_term, nc, C.s));
  }
  const long long hoff = m->cfg.tie_embeddings ? C.Lo.tok : C.Lo.head;
  for (int i = 0; i < noff; ++i) {
    // offset_projs[k] = Linear -> GELU -> Linear, then the (tied) head
    cg_gemm_desc g = lin_fwd(C, A.xf, d, C.Lo.off1w[i], d, d, d, A.og[i], d);
    g.epilogue = CG_EPI_BIAS | CG_EPI_GELU | CG_EPI_GELU_DERIV; g.bias = P(C, C.Lo.off1b[i]);
    g.aux_out = A.oa[i]; g.ld_aux = d;
    CK(cg_gemm(&g, C.s));
    g = lin_fwd(C, A.og[i], d, C.Lo.off2w[i], d, d, d, A.opj[i], d);
    g.epilogue = CG_EPI_BIAS; g.bias = P(C, C.Lo.off2b[i]);
    CK(cg_gemm(&g, C.s));
    g = lin_fwd(C, A.opj[i], d, hoff, d, ld_off >= D.Vp ? D.Vp : D.V, d, offset_logits[i], ld_off);
    g.c_dtype = CG_F32;
    CK(cg_gemm(&g, C.s));
  }
  m->aux_ready = 1;
  return CG_OK;
}

namespace {
// the embedding backward (model_tiny_gpt.py:305-312): tok_emb (+ pos_emb) gradients from the
// residual gradient A.g left by block 0's first LayerNorm backward
int embed_backward(const Ctx& C, cg_model* m, uint32_t seed, float p, int accumulate) {
  const Dims& D = C.D;
  const Acts& A = C.A;
  const int d = D.d;
  // tied tok_emb already holds the head contribution from phase 0 -> always accumulate
  const int acc_tok = m->cfg.tie_embeddings ? 1 : accumulate;
  CK(cg_embed_bwd(m->idx, A.g, G(C, C.Lo.tok), nullptr, C.B, C.T, D.V, d, site_seed(seed, -1, SITE_EMB), p, acc_tok,
                  A.embws, A.nb.embws, C.s));
  if (C.Lo.pos >= 0)
    CK(cg_embed_bwd(m->idx, A.g, nullptr, G(C, C.Lo.pos), C.B, C.T, D.V, d, site_seed(seed, -1, SITE_EMB), p,
                    accumulate, A.embws, A.nb.embws, C.s));
  return CG_OK;
}
}  // namespace

extern "C" int cg_model_backward(cg_model* m, int phase, int layer, int accumulate, void* stream) {
  if (!m || !m->idx || !m->grads) return CG_EINVAL;
  Ctx C;
  CK(make_ctx(m, m->B, m->T, stream, C));
  const Dims& D = C.D;
  const Acts& A = C.A;
  const int d = D.d;
  const long long M = C.M;
  const float p = train_p(m);
  const float eps = m->cfg.ln_eps > 0 ? m->cfg.ln_eps : 1e-5f;
  const uint32_t seed = m->seed;

  if (phase == 0) {
    pending(m).n = 0;  // a backward starts here: drop anything an abandoned one left
    CK(transpose_weights(C));  // this step's shadow weights -> K-contiguous dX operands
    const long long hoff = m->cfg.tie_embeddings ? C.Lo.tok : C.Lo.head;
    CK(fill_head2(C, hoff));
    if (m->targets && m->head_grad_scale_dev)  // d(objective)/d(loss) still on the device
      CK(cg_scale_dev(C.dt == CG_BF16 ? CG_BF16X2 : C.dt, A.dlogits, A.ldl, (int)M, D.Vp, m->head_grad_scale_dev,
                      C.s));
    m->head_dw_pending = 0;
    if (m->targets) {
      // d(head weight) = s dlogits^T . xf: deferred into the first dW group when nothing else
      // adds into it before that launch (the aux heads do, and reuse dlogits)
      if (!m->cfg.opts.head_dw_separate && C.dt == CG_BF16 && D.L > 0 && m->cfg.tie_embeddings && !m->cfg.termination_aux &&
          m->cfg.n_offsets <= 0)
      {
        m->head_dw_off = hoff;
        m->head_dw_alpha = m->head_grad_scale;
        m->head_dw_accumulate = accumulate;
        m->head_dw_pending = 1;
      }
      else
        CK(head_dw_now(C, hoff, m->head_grad_scale, accumulate));
      // dxf = s dlogits . E
      cg_gemm_desc g = head_dx(C, hoff, A.dtmp, d);
      g.c_dtype = CG_F32;
      g.alpha = m->head_grad_scale;
      CK(cg_gemm(&g, C.s));
    } else {
      // no next-codon loss (aux-only objective, e.g. a replay batch): nothing to scale
      if (m->head_grad_scale != 0.f || !m->aux_ready) return CG_EINVAL;
      if (!accumulate) CK(zero_grad(C, hoff, (long long)D.Vp * d));
      if (hipMemsetAsync(A.dtmp, 0, (size_t)M * d * 4, C.s) != hipSuccess) return CG_ELAUNCH;
    }
    CK(aux_backward(C, accumulate));  // aux heads add into d(head) and dxf
    float* xL = A.x + (size_t)D.L * M * d;
    const int ll = D.L - 1;
    // gT feeds block L-1's MLP output Linear: its bias gradient (GELU mode) is gT's column sum
    float* db2 = (D.L > 0 && !D.swiglu) ? G(C, C.Lo.lay[ll].b2) : nullptr;
    m->dw_done_layer = D.L;
    CK(cg_layernorm_bwd(CG_F32, A.dtmp, d, xL, d, A.meanf, A.rstdf, P(C, C.Lo.lnfw), nullptr, A.g, C.dt,
                        D.L > 0 ? A.slot[slot_of(D, ll)].gin : nullptr, site_seed(seed, ll, SITE_MLP), D.L > 0 ? p : 0.f, A.lnpart,
                        A.nb.lnp, G(C, C.Lo.lnfw), G(C, C.Lo.lnfb), db2, accumulate, (int)M, d, eps, C.s));
    CK(flush_reduce(m, C.s));  // the aux heads' bias gradients (their bucket is complete here)
    return CG_OK;
  }
  if (phase == 1) {
    const int l = layer;
    if (l < 0 || l >= D.L) return CG_EINVAL;
    const auto& o = C.Lo.lay[l];
    const auto& a = A.la[l];
    float* xl = A.x + (size_t)l * M * d;
    const DwSlot& sl = A.slot[slot_of(D, l)];
    // ---------------- MLP branch: sl.gin = dL/d(mlp out) (dropout mask applied); the weight
    // gradients of the block are produced by its group's flush_dw from the slot operands
    if (!D.swiglu) {
      // (b2's gradient was produced by the LayerNorm backward that wrote gin)
      // dGELU product.  fc1's bias gradient: the column sums of dH, taken by the block's grouped dW
      // launch from the dH fragments it streams anyway (round 6; the dGELU epilogue's column sums
      // cost this product 16-22 us per layer at C4), or -- when that launch splits the tokens --
      // by this product's fused column-sum epilogue (64-row partials)
      const bool in_dw = fc1_bias_in_dw(C, l);
      cg_gemm_desc g = lin_dx(C, sl.gin, d, o.w2, D.hid, d, D.hid, sl.dmlp, D.hid, a.w2T);
      g.epilogue = CG_EPI_DGELU | CG_EPI_GELU_DERIV | (in_dw ? 0 : CG_EPI_COLSUM); g.aux = a.a; g.ld_aux = D.hid;
      if (!in_dw) {
        g.workspace = sl.cpart;
        g.ws_bytes = A.nb.cpart;
      }
      CK(cg_gemm(&g, C.s));
      if (!in_dw) CK(defer_reduce(m, sl.cpart, D.hid, (int)((M + 63) / 64), D.hid, G(C, o.b1), accumulate, C.s));
      g = lin_dx(C, sl.dmlp, D.hid, o.w1, d, D.hid, d, A.dsmall, d, a.w1T);  // dL/d(ln2 out), compute dtype
      CK(cg_gemm(&g, C.s));
    } else {
      // dL/ds product with the SwiGLU backward in its epilogue (d(gate|up) straight to dmlp)
      cg_gemm_desc g = lin_dx(C, sl.gin, d, o.wd, D.Hp, d, D.Hp, sl.dmlp, 2 * D.Hp, a.wdT);
      g.epilogue = CG_EPI_DSWIGLU; g.aux = a.gu; g.ld_aux = 2 * D.Hp; g.n_valid = D.hid;
      int rc = C.dt == CG_BF16 ? cg_gemm(&g, C.s) : CG_EUNSUPPORTED;
      if (rc == CG_EUNSUPPORTED) {
        g = lin_dx(C, sl.gin, d, o.wd, D.Hp, d, D.Hp, A.dsmall, D.Hp, a.wdT);
        CK(cg_gemm(&g, C.s));
        rc = cg_swiglu_bwd(C.dt, a.gu, 2 * D.Hp, D.Hp, A.dsmall, D.Hp, sl.dmlp, 2 * D.Hp, (int)M, D.hid, C.s);
      }
      CK(rc);
      g = lin_dx(C, sl.dmlp, 2 * D.Hp, o.wgu, d, 2 * D.Hp, d, A.dsmall, d, a.wguT);
      CK(cg_gemm(&g, C.s));
    }
    // gattn = dL/d(proj out); its column sum is the proj bias gradient
    CK(ln_bwd_deferred(C, C.dt, A.dsmall, a.xmid, a.mean2, a.rstd2, o.ln2w, A.g, sl.gattn, 0, 0.f, sl.lnp2,
                       G(C, o.ln2w), G(C, o.ln2b), G(C, o.bp), accumulate));
    // ---------------- attention branch
    cg_gemm_desc g = lin_dx(C, sl.gattn, d, o.wp, d, d, d, A.dsmall, d, a.pT);
    CK(cg_gemm(&g, C.s));
    // the qkv bias gradient = column sums of the (un-rotated) dqkv: produced by the MFMA attention
    // backward itself as per-tile partials (with RoPE it rotates dQ / dK back before the stores and
    // the partials), else a colsum pass after the vector kernels and the table inverse rotation
    const void* segp = m->cfg.sep_id >= 0 ? A.seg : nullptr;
    const void* dmask_b = p > 0.f ? a.dmask : nullptr;
    const bool rope_in = D.rope && !m->cfg.opts.rope_tables;  // the inverse rotation inside the kernels
    const float* rc_cos = rope_in ? m->rope_cos : nullptr;
    const float* rc_sin = rope_in ? m->rope_sin : nullptr;
    int rc = CG_EUNSUPPORTED;
    if (!D.rope || rope_in)
      rc = cg_attn_bwd_algo(m->cfg.opts.attn_bwd_algo, C.dt, a.qkv, D.Nqkv, (const int32_t*)segp, a.y, d, A.dsmall,
                            d, a.lse, sl.dqkv, D.Nqkv, C.B, C.T, D.H, D.KV, D.hd, m->window,
                            site_seed(seed, l, SITE_ATTN), p, dmask_b, sl.bpart, D.Nqkv, rc_cos, rc_sin, A.delta,
                            A.nb.delta, C.s);
    const bool fused_bias = rc == CG_OK;
    if (rc == CG_EUNSUPPORTED) {
      rc = cg_attn_bwd(C.dt, a.qkv, D.Nqkv, (const int32_t*)segp, a.y, d, A.dsmall, d, a.lse, sl.dqkv, D.Nqkv, C.B,
                       C.T, D.H, D.KV, D.hd, m->window, site_seed(seed, l, SITE_ATTN), p, dmask_b, nullptr, 0,
                       A.delta, A.nb.delta, C.s);
      if (rc == CG_OK && D.rope)
        rc = cg_rope_tab(C.dt, sl.dqkv, D.Nqkv, C.B, C.T, D.H, D.KV, D.hd, m->rope_cos, m->rope_sin, 1, C.s);
    }
    CK(rc);
    if (fused_bias)
      CK(defer_reduce(m, sl.bpart, D.Nqkv, C.B * ((C.T + 127) / 128), D.Nqkv, G(C, o.bqkv), accumulate, C.s));
    else
      CK(bias_grad(C, sl.dqkv, D.Nqkv, D.Nqkv, o.bqkv, accumulate));
    g = lin_dx(C, sl.dqkv, D.Nqkv, o.wqkv, d, D.Nqkv, d, A.dsmall, d, a.qkvT);  // dL/d(ln1 out)
    CK(cg_gemm(&g, C.s));
    // the group's weight gradients once its lowest block is done.  (The last group on a side
    // stream beside block 0's LayerNorm backward and the embedding backward measured slower on
    // every config, round 4: the persistent walker loses CUs to the streaming kernels.)
    if (group_ends(D, l)) {
      CK(flush_dw(C, l + slot_of(D, l), l, accumulate));
      m->dw_done_layer = l;
    }
    // block l-1's MLP output gradient (its bias grad fused as above; it lands in block l-1's
    // gradient range, which is final only after block l-1's group)
    float* db2 = (l > 0 && !D.swiglu) ? G(C, C.Lo.lay[l - 1].b2) : nullptr;
    CK(ln_bwd_deferred(C, C.dt, A.dsmall, xl, a.mean1, a.rstd1, o.ln1w, A.g,
                       l > 0 ? A.slot[slot_of(D, l - 1)].gin : nullptr, site_seed(seed, l - 1, SITE_MLP),
                       l > 0 ? p : 0.f, sl.lnp1, G(C, o.ln1w), G(C, o.ln1b), db2, accumulate));
    // the group's parameter-gradient reductions (its LayerNorms, fused biases) in one launch,
    // before the caller starts the group's bucket all-reduce
    if (group_ends(D, l)) CK(flush_reduce(m, C.s));
    return CG_OK;
  }
  if (phase == 2) {
    CK(flush_reduce(m, C.s));  // nothing is pending after block 0; kept for partial phase sequences
    if (m->head_dw_pending) {  // a partial phase sequence: no dW group took the head's product
      m->head_dw_pending = 0;
      CK(head_dw_now(C, m->head_dw_off, m->head_dw_alpha, m->head_dw_accumulate));
    }
    CK(embed_backward(C, m, seed, p, accumulate));
    return CG_OK;
  }
  return CG_EINVAL;
}

// attention probabilities of block `layer` of the last forward (fp32 [B][H][T][T])
extern "C" int cg_model_attn_probs(const cg_model* m, int layer, float* out, void* stream) {
  if (!m || !out) return CG_EINVAL;
  Ctx C;
  CK(make_ctx(m, m->B, m->T, stream, C));
  if (layer < 0 || layer >= C.D.L) return CG_EINVAL;
  const auto& a = C.A.la[layer];
  return cg_attn_probs(C.dt, a.qkv, C.D.Nqkv, m->cfg.sep_id >= 0 ? C.A.seg : nullptr, a.lse, out, C.B, C.T, C.D.H,
                       C.D.KV, C.D.hd, m->window, C.s);
}

extern "C" const void* cg_model_hidden(const cg_model* m, int which, int* dtype_out, long long* ld) {
  if (!m) return nullptr;
  Ctx C;
  if (make_ctx(m, m->B, m->T, nullptr, C) != CG_OK) return nullptr;
  const long long M = C.M;
  if (ld) *ld = C.D.d;
  if (which >= 0 && which <= C.D.L) {
    if (dtype_out) *dtype_out = CG_F32;
    return C.A.x + (size_t)which * M * C.D.d;
  }
  if (which == C.D.L + 1) {
    if (dtype_out) *dtype_out = C.dt;
    return C.A.xf;
  }
  return nullptr;
}

// ===========================================================================
// Incremental decoding (KV cache)
// ===========================================================================
extern "C" int cg_attn_decode(int dtype, const void* q, long long ldq, const void* cache, long long ldc, int Tmax,
                              int pos, const int32_t* segstate, int window, int B, int H, int KV, int hd, void* y,
                              long long ldy, void* stream);
extern "C" int cg_segstate_step(const int64_t* tok, int B, int sep_id, int pos, int32_t* segstate, void* stream);

namespace {
struct DecWS {
  float *x, *xmid, *mean, *rstd;
  void *h, *qkv, *y, *a, *g, *gu, *s, *xf;
};
size_t carve_dec(const cg_model_cfg* c, const Dims& D, int B, char* base, DecWS& W) {
  WS w{base, 0};
  const size_t es = c->dtype == CG_BF16 ? 2 : 4;
  const int d = D.d;
  W.x = w.take<float>((size_t)B * d * 4);
  W.xmid = w.take<float>((size_t)B * d * 4);
  W.mean = w.take<float>((size_t)B * 4);
  W.rstd = w.take<float>((size_t)B * 4);
  W.h = w.take<char>((size_t)B * d * es);
  W.qkv = w.take<char>((size_t)B * D.Nqkv * es);
  W.y = w.take<char>((size_t)B * d * es);
  W.a = W.g = W.gu = W.s = nullptr;
  if (!D.swiglu) {
    W.a = w.take<char>((size_t)B * D.hid * es);
    W.g = w.take<char>((size_t)B * D.hid * es);
  } else {
    W.gu = w.take<char>((size_t)B * 2 * D.Hp * es);
    W.s = w.take<char>((size_t)B * D.Hp * es);
  }
  W.xf = w.take<char>((size_t)B * d * es);
  return w.off + 256;
}
// a Ctx whose row count is the B decoding rows (no activation workspace)
int make_dec_ctx(const cg_model* m, int B, void* stream, Ctx& C) {
  if (!dims_of(&m->cfg, C.D)) return CG_EINVAL;
  build_layout(&m->cfg, C.D, C.Lo);
  C.m = m;
  C.B = B; C.T = 1; C.M = B;
  C.dt = m->cfg.dtype;
  C.s = (hipStream_t)stream;
  return CG_OK;
}
}  // namespace

extern "C" size_t cg_kv_cache_bytes(const cg_model_cfg* cfg, int B, int Tmax) {
  Dims D;
  if (!dims_of(cfg, D) || B <= 0 || Tmax <= 0) return 0;
  const size_t es = cfg->dtype == CG_BF16 ? 2 : 4;
  return (size_t)D.L * B * Tmax * 2 * D.kvd * es;
}

extern "C" size_t cg_decode_workspace_bytes(const cg_model_cfg* cfg, int B) {
  Dims D;
  if (!dims_of(cfg, D) || B <= 0) return 0;
  DecWS W;
  return carve_dec(cfg, D, B, nullptr, W);
}

extern "C" int cg_model_prefill(cg_model* m, const int64_t* idx, int B, int T, int window, void* cache, int Tmax,
                                int32_t* segstate, float* logits, void* stream) {
  if (!m || !idx || !cache || !segstate || B <= 0 || T <= 0 || Tmax < T || Tmax > m->cfg.block_size) return CG_EINVAL;
  CK(cg_model_forward(m, idx, nullptr, B, T, 0, 0, window, logits, nullptr, stream));
  Ctx C;
  CK(make_ctx(m, B, T, stream, C));
  const Dims& D = C.D;
  const size_t es = C.dt == CG_BF16 ? 2 : 4;
  const size_t row = (size_t)2 * D.kvd * es;
  // the [k|v] columns of each qkv row (post-RoPE K) -> cache rows 0..T-1, one T-row 2-D copy per
  // (layer, sequence)
  for (int l = 0; l < D.L; ++l)
    for (int b = 0; b < B; ++b) {
      const char* src = (const char*)C.A.la[l].qkv + ((size_t)b * T * D.Nqkv + D.d) * es;
      char* dst = (char*)cache + ((size_t)l * B + b) * Tmax * row;
      if (hipMemcpy2DAsync(dst, row, src, (size_t)D.Nqkv * es, row, T, hipMemcpyDeviceToDevice, C.s) != hipSuccess)
        return CG_ELAUNCH;
    }
  if (m->cfg.sep_id >= 0) {
    if (hipMemcpy2DAsync(segstate, 4, C.A.seg + (T - 1), (size_t)T * 4, 4, B, hipMemcpyDeviceToDevice, C.s) !=
        hipSuccess)
      return CG_ELAUNCH;
  } else if (hipMemsetAsync(segstate, 0, (size_t)B * 4, C.s) != hipSuccess) {
    return CG_ELAUNCH;
  }
  return CG_OK;
}

extern "C" int cg_model_decode(cg_model* m, const int64_t* tok, int B, int pos, void* cache, int Tmax,
                               int32_t* segstate, void* dec_ws, size_t dec_ws_bytes, float* logits, void* stream) {
  if (!m || !tok || !cache || !segstate || !dec_ws || !logits || B <= 0) return CG_EINVAL;
  if (pos < 0 || pos >= Tmax || Tmax > m->cfg.block_size) return CG_EINVAL;
  if (m->cfg.dtype == CG_BF16 && !m->shadow) return CG_EINVAL;
  if (m->cfg.use_rope && (!m->rope_cos || !m->rope_sin)) return CG_EINVAL;
  Ctx C;
  CK(make_dec_ctx(m, B, stream, C));
  const Dims& D = C.D;
  DecWS W;
  if (carve_dec(&m->cfg, D, B, nullptr, W) > dec_ws_bytes) return CG_EINVAL;
  carve_dec(&m->cfg, D, B, (char*)dec_ws, W);
  const int d = D.d;
  const float eps = m->cfg.ln_eps > 0 ? m->cfg.ln_eps : 1e-5f;
  const size_t es = C.dt == CG_BF16 ? 2 : 4;
  const size_t row = (size_t)2 * D.kvd * es;
  CK(cg_embed_fwd(tok, P(C, C.Lo.tok), C.Lo.pos >= 0 ? P(C, C.Lo.pos) + (size_t)pos * d : nullptr, W.x, B, 1, d, 0,
                  0.f, C.s));
  CK(cg_segstate_step(tok, B, m->cfg.sep_id, pos, segstate, C.s));
  for (int l = 0; l < D.L; ++l) {
    const auto& o = C.Lo.lay[l];
    CK(cg_layernorm_fwd(C.dt, W.x, d, P(C, o.ln1w), P(C, o.ln1b), W.h, d, W.mean, W.rstd, B, d, eps, C.s));
    cg_gemm_desc g = lin_fwd(C, W.h, d, o.wqkv, d, D.Nqkv, d, W.qkv, D.Nqkv);
    g.epilogue = CG_EPI_BIAS; g.bias = P(C, o.bqkv);
    CK(cg_gemm(&g, C.s));
    if (D.rope)
      CK(cg_rope_tab(C.dt, W.qkv, D.Nqkv, B, 1, D.H, D.KV, D.hd, m->rope_cos + (size_t)pos * (D.hd / 2),
                     m->rope_sin + (size_t)pos * (D.hd / 2), 0, C.s));
    char* cl = (char*)cache + (size_t)l * B * Tmax * row;
    if (hipMemcpy2DAsync(cl + (size_t)pos * row, (size_t)Tmax * row, (const char*)W.qkv + (size_t)d * es,
                         (size_t)D.Nqkv * es, row, B, hipMemcpyDeviceToDevice, C.s) != hipSuccess)
      return CG_ELAUNCH;
    CK(cg_attn_decode(C.dt, W.qkv, D.Nqkv, cl, 2 * D.kvd, Tmax, pos, m->cfg.sep_id >= 0 ? segstate : nullptr,
                      m->window, B, D.H, D.KV, D.hd, W.y, d, C.s));
    g = lin_fwd(C, W.y, d, o.wp, d, d, d, W.xmid, d);
    g.c_dtype = CG_F32;
    g.epilogue = CG_EPI_BIAS | CG_EPI_RESID; g.bias = P(C, o.bp); g.resid = W.x; g.ldr = d;
    CK(cg_gemm(&g, C.s));
    CK(cg_layernorm_fwd(C.dt, W.xmid, d, P(C, o.ln2w), P(C, o.ln2b), W.h, d, W.mean, W.rstd, B, d, eps, C.s));
    if (!D.swiglu) {
      g = lin_fwd(C, W.h, d, o.w1, d, D.hid, d, W.g, D.hid);
      g.epilogue = CG_EPI_BIAS | CG_EPI_GELU | CG_EPI_GELU_DERIV; g.bias = P(C, o.b1); g.aux_out = W.a; g.ld_aux = D.hid;
      CK(cg_gemm(&g, C.s));
      g = lin_fwd(C, W.g, D.hid, o.w2, D.hid, d, D.hid, W.x, d);
      g.c_dtype = CG_F32;
      g.epilogue = CG_EPI_BIAS | CG_EPI_RESID; g.bias = P(C, o.b2); g.resid = W.xmid; g.ldr = d;
      CK(cg_gemm(&g, C.s));
    } else {
      g = lin_fwd(C, W.h, d, o.wgu, d, 2 * D.Hp, d, W.gu, 2 * D.Hp);
      CK(cg_gemm(&g, C.s));
      CK(cg_swiglu_fwd(C.dt, W.gu, 2 * D.Hp, D.Hp, W.s, D.Hp, B, D.hid, C.s));
      g = lin_fwd(C, W.s, D.Hp, o.wd, D.Hp, d, D.Hp, W.x, d);
      g.c_dtype = CG_F32;
      g.epilogue = CG_EPI_RESID; g.resid = W.xmid; g.ldr = d;
      CK(cg_gemm(&g, C.s));
    }
  }
  CK(cg_layernorm_fwd(C.dt, W.x, d, P(C, C.Lo.lnfw), P(C, C.Lo.lnfb), W.xf, d, W.mean, W.rstd, B, d, eps, C.s));
  const long long hoff = m->cfg.tie_embeddings ? C.Lo.tok : C.Lo.head;
  cg_gemm_desc g = lin_fwd(C, W.xf, d, hoff, d, D.V, d, logits, D.V);
  g.c_dtype = CG_F32;
  CK(cg_gemm(&g, C.s));
  return CG_OK;
}

extern "C" size_t cg_struct_bytes(const char* name) {
  if (!name) return 0;
  const std::string n(name);
#define CG_SZ(T) \
  if (n == #T) return sizeof(T);
  CG_SZ(cg_gemm_desc) CG_SZ(cg_dw_product) CG_SZ(cg_dw_group) CG_SZ(cg_reduce_job) CG_SZ(cg_reduce_batch)
  CG_SZ(cg_transpose_item) CG_SZ(cg_transpose_batch) CG_SZ(cg_adamw_segment) CG_SZ(cg_model_cfg)
  CG_SZ(cg_param_entry) CG_SZ(cg_model) CG_SZ(cg_model_opts)
#undef CG_SZ
  return 0;
}

extern "C" const char* cg_version(void) { return "codonlm_hip 0.5 gfx950"; }
