// api.hip -- C ABI entry points (include/uthot.h) and the host-side space
// compiler.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "ut_internal.h"

namespace ut {

int set_err(ut_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// device allocation accounting: pointer -> (bytes, device), process-wide
namespace {
std::mutex g_mem_mu;
std::unordered_map<void*, std::pair<size_t, int>> g_mem_ptrs;
std::unordered_map<int, int64_t> g_mem_bytes;
}  // namespace

hipError_t dmalloc(void** p, size_t bytes) {
  const hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return e;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(g_mem_mu);
  g_mem_ptrs[*p] = {bytes, dev};
  g_mem_bytes[dev] += (int64_t)bytes;
  return e;
}

void dfree(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> g(g_mem_mu);
    auto it = g_mem_ptrs.find(p);
    if (it != g_mem_ptrs.end()) {
      g_mem_bytes[it->second.second] -= (int64_t)it->second.first;
      g_mem_ptrs.erase(it);
    }
  }
  (void)hipFree(p);
}

void mark(ut_ctx* c, const char* name) {
  if (!c->timing.on) return;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return;
  hipEventRecord(e, c->stream);
  c->timing.marks.push_back({name, c->stream, e, c->timing.round});
}

static void timing_begin(ut_ctx* c) {
  if (!c->timing.on) return;
  ++c->timing.round;
  c->timing.in_round = true;
  mark(c, "");
}

static int timing_end(ut_ctx* c) {
  c->timing.in_round = false;
  return 0;
}

// read every recorded event into the per-stage totals (one host sync)
static int timing_collect(ut_ctx* c, bool keep) {
  auto& T = c->timing;
  if (T.marks.empty()) return 0;
  UT_HIP(c, ut::sync_all(c));
  for (size_t i = 0; keep && i < T.marks.size(); ++i) {
    const auto& m = T.marks[i];
    if (m.name.empty()) {
      // a round's first mark: the time since the previous round's last mark on
      // its stream is "between" (the device idle or finishing unmarked work
      // while the host is between the two rounds)
      if (i == 0 || T.marks[i - 1].round == m.round) continue;
      for (size_t j = i; j-- > 0;) {
        if (T.marks[j].round != m.round - 1) break;
        if (T.marks[j].stream != m.stream) continue;
        float ms = 0.f;
        hipEventElapsedTime(&ms, T.marks[j].ev, m.ev);
        auto it = T.totals.begin();
        while (it != T.totals.end() && it->first != "between") ++it;
        if (it == T.totals.end()) T.totals.push_back({"between", {0.0, 0}}), it = T.totals.end() - 1;
        it->second.first += ms;
        it->second.second += 1;
        break;
      }
      continue;
    }
    for (size_t j = i; j-- > 0;) {  // the previous mark of the same round on the same stream
      if (T.marks[j].round != m.round) break;
      if (T.marks[j].stream != m.stream) continue;
      float ms = 0.f;
      hipEventElapsedTime(&ms, T.marks[j].ev, m.ev);
      auto it = T.totals.begin();
      while (it != T.totals.end() && it->first != m.name) ++it;
      if (it == T.totals.end()) T.totals.push_back({m.name, {0.0, 0}}), it = T.totals.end() - 1;
      it->second.first += ms;
      it->second.second += 1;
      break;
    }
  }
  for (auto& m : T.marks) hipEventDestroy(m.ev);
  T.marks.clear();
  return 0;
}

static void free_space(Space& s) {
  if (s.d_params) ut::dfree(s.d_params);
  if (s.d_order) ut::dfree(s.d_order);
  if (s.d_words) ut::dfree(s.d_words);
  if (s.d_block_last) ut::dfree(s.d_block_last);
  if (s.d_lut) ut::dfree(s.d_lut);
  if (s.d_vtab) ut::dfree(s.d_vtab);
  for (void* q : {(void*)s.d_order_col, (void*)s.d_perm_params, (void*)s.d_perm_bytes, (void*)s.d_perm_off,
                  (void*)s.d_perm_offbase, (void*)s.d_perm_len, (void*)s.d_comp,
                  (void*)s.d_col_param, (void*)s.d_cat_ccol, (void*)s.d_num_feat, (void*)s.d_feat_num})
    if (q) ut::dfree(q);
  s = Space();
}

// Build the fixed outer message of hash_config (manipulator.py:233-243):
//   for i, p in enumerate(sorted params): name ++ hash_value ++ str(i) ++ "|"
// with hash_value = "b'" hex "'" (py3, primitive) or hex.
static int compile_hash_layout(ut_ctx* c, const std::vector<std::string>& names,
                               const std::vector<bool>& primitive) {
  Space& s = c->space;
  const int32_t P = s.P;
  std::vector<uint8_t> msg;
  std::vector<int64_t> hole_start(P);
  for (int32_t j = 0; j < P; ++j) {
    const int32_t p = s.host_order[j];
    msg.insert(msg.end(), names[p].begin(), names[p].end());
    const bool wrap = primitive[p] && !s.py2;
    if (wrap) { msg.push_back('b'); msg.push_back('\''); }
    hole_start[j] = (int64_t)msg.size();
    for (int q = 0; q < 64; ++q) msg.push_back(0);
    if (wrap) msg.push_back('\'');
    const std::string idx = std::to_string(j);
    msg.insert(msg.end(), idx.begin(), idx.end());
    msg.push_back('|');
  }
  const int64_t L = (int64_t)msg.size();
  msg.push_back(0x80);
  while (msg.size() % 64 != 56) msg.push_back(0);
  const uint64_t bits = (uint64_t)L * 8;
  for (int q = 7; q >= 0; --q) msg.push_back((uint8_t)(bits >> (8 * q)));
  const int64_t NBLK = (int64_t)msg.size() / 64;
  // a 4-byte word must never touch two holes (the kernel fetches one hole per word)
  for (int32_t q = 0; q + 1 < P; ++q)
    UT_CHECK(c, hole_start[q + 1] - (hole_start[q] + 64) >= 3, UT_EUNSUPPORTED,
             "hash layout: parameter names too short to separate the digest holes");
  std::vector<HashWord> words(NBLK * 16);
  std::vector<int32_t> block_last(NBLK);
  int32_t j = 0;  // first hole that may overlap the current word
  int32_t running = -1;
  for (int64_t w = 0; w < NBLK * 16; ++w) {
    HashWord hw;
    hw.tmpl = ((uint32_t)msg[4 * w] << 24) | ((uint32_t)msg[4 * w + 1] << 16) | ((uint32_t)msg[4 * w + 2] << 8) |
              (uint32_t)msg[4 * w + 3];
    hw.info = 0;
    while (j < P && hole_start[j] + 64 <= 4 * w) ++j;
    if (j < P && hole_start[j] < 4 * w + 4 && hole_start[j] + 64 > 4 * w) {
      const int64_t d = 4 * w - hole_start[j];           // -3 .. 63
      const int64_t q = (d >= 0) ? d / 4 : -1;           // floor(d / 4): hex word holding byte d
      const uint32_t slot = (uint32_t)(j & 1) * 16;      // hole j lives in hex slot j % 2
      uint32_t info = HW_HOLE | ((uint32_t)(d - 4 * q) * 8) << HW_SHIFT_POS;
      if (q >= 0) info |= HW_LO_VALID | (slot + (uint32_t)q);
      if (q + 1 < 16) info |= HW_HI_VALID | ((slot + (uint32_t)(q + 1)) << HW_HI_POS);
      hw.info = info;
      if (j > running) running = j;
    }
    words[w] = hw;
    if (w % 16 == 15) block_last[w / 16] = running;
  }
  s.outer_len = L;
  s.outer_blocks = NBLK;
  UT_HIP(c, ut::dmalloc((void**)&s.d_words, sizeof(HashWord) * words.size()));
  UT_HIP(c, hipMemcpy(s.d_words, words.data(), sizeof(HashWord) * words.size(), hipMemcpyHostToDevice));
  UT_HIP(c, ut::dmalloc((void**)&s.d_block_last, sizeof(int32_t) * block_last.size()));
  UT_HIP(c, hipMemcpy(s.d_block_last, block_last.data(), sizeof(int32_t) * block_last.size(), hipMemcpyHostToDevice));
  return 0;
}

static int history_alloc(ut_ctx* c, int64_t cap) {
  int64_t p2 = 1024;
  while (p2 < cap) p2 <<= 1;
  if (c->hist_keys) {
    UT_HIP(c, ut::sync_all(c));
    ut::dfree(c->hist_keys);
    ut::dfree(c->hist_state);
  }
  UT_HIP(c, ut::dmalloc((void**)&c->hist_keys, sizeof(uint32_t) * 8 * p2));
  UT_HIP(c, ut::dmalloc((void**)&c->hist_state, sizeof(uint32_t) * p2));
  UT_HIP(c, hipMemsetAsync(c->hist_state, 0, sizeof(uint32_t) * p2, c->stream));
  c->hist_cap = p2;
  c->hist_count = 0;
  return 0;
}

}  // namespace ut

using namespace ut;

extern "C" {

int ut_version(void) { return 1; }

int ut_device_bytes(int32_t device, int64_t* bytes) {
  if (!bytes) return UT_EINVAL;
  std::lock_guard<std::mutex> g(g_mem_mu);
  auto it = g_mem_bytes.find(device);
  *bytes = it == g_mem_bytes.end() ? 0 : it->second;
  return 0;
}


int ut_ctx_create(int device, uint64_t seed, ut_ctx** out) {
  if (!out) return UT_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return UT_EHIP;
  if (hipSetDevice(device) != hipSuccess) return UT_EHIP;
  ut_ctx* c = new ut_ctx();
  c->device = device;
  c->seed = seed;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu >= 8)
    c->n_cu = ncu;
  int lds = 0;
  if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lds > 0)
    c->max_lds = (size_t)lds;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->fit_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fit, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_prefit, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fit_x, hipEventDisableTiming) != hipSuccess) {
    ut_ctx_destroy(c);
    return UT_EHIP;
  }
  c->stream = c->own_stream;
  // ut_comm_bcast_results' count / agreement words: allocated with the
  // context, so no allocation can fail between a rank's entry into
  // ut_comm_init and its first collective
  if (ut::ensure(c, c->cm_cnt, 2)) {
    ut_ctx_destroy(c);
    return UT_ENOMEM;
  }
  if (const char* e = getenv("UT_CHOL_FUSE")) c->chol_fuse = atoi(e);
  if (const char* e = getenv("UT_TRINV_BIG")) c->trinv_big = atoi(e);
  if (const char* e = getenv("UT_CHOL_MERGED")) c->chol_merged = atoi(e);
  // the fit kernels' waves at s_setprio 3 (gp.hip g_fit_prio): beside the
  // round's hash grid their instructions go first
  if (ut::set_fit_prio(1)) {
    ut_ctx_destroy(c);
    return UT_EHIP;
  }
  if (const char* e = getenv("UT_VAR_SPLIT")) c->var_split = atoi(e) != 0;
  if (const char* e = getenv("UT_DE_AOS")) c->de_aos = atoi(e) != 0;
  if (const char* e = getenv("UT_HASH_WG_PER_CU")) c->hash_wg_per_cu = atoi(e);
  if (const char* e = getenv("UT_CAT_KSTAR")) c->cat_enable = atoi(e) != 0;
  if (const char* e = getenv("UT_FIT_DEFER")) c->fit_defer = atoi(e) != 0;
  if (const char* e = getenv("UT_KSTAR_Q")) c->kstar_q = atoi(e) != 0;
  *out = c;
  return 0;
}

int ut_ctx_destroy(ut_ctx* c) {
  if (!c) return UT_EINVAL;
  hipSetDevice(c->device);
  if (c->stream) ut::sync_all(c);
  ut::comm_release(c);
  free_space(c->space);
  auto fr = [](void* p) { if (p) ut::dfree(p); };
  fr(c->pop); fr(c->pso_vel); fr(c->pso_best);
  fr(c->pop_dig); fr(c->pop_aos);
  for (size_t s = 0; s < c->pop_slots.size(); ++s) {
    if ((int32_t)s == c->pop_slot) continue;   // the selected slot's buffers are the fields above
    fr(c->pop_slots[s].pop); fr(c->pop_slots[s].pso_vel); fr(c->pop_slots[s].pso_best); fr(c->pop_slots[s].pop_dig);
    fr(c->pop_slots[s].pop_aos);
  }
  fr(c->r_mask.p); fr(c->r_fresh.p); fr(c->r_pairs.p); fr(c->r_npairs.p); fr(c->de_xbits.p); fr(c->par_dig.p);
  fr(c->hs_mask.p); fr(c->hs_fresh.p);
  fr(c->pr_mu.p); fr(c->pr_ub.p); fr(c->pr_score.p); fr(c->pr_mpart.p); fr(c->pr_kst.p); fr(c->pr_vpart.p);
  fr(c->pr_idx.p); fr(c->pr_count.p); fr(c->pr_ucand.p); fr(c->pr_cnorm.p);
  fr(c->pr_k2.p); fr(c->pr_f2.p); fr(c->pr_exact.p); fr(c->app_ws.p); fr(c->var_vbuf.p);
  fr(c->hist_keys); fr(c->hist_state); fr(c->batch_slots);
  fr(c->gp_Xs); fr(c->gp_xnorm); fr(c->gp_K); fr(c->gp_Linv); fr(c->gp_y); fr(c->gp_tmp);
  fr(c->gp_alpha); fr(c->gp_beta); fr(c->gp_inv_ell); fr(c->gp_stats); fr(c->gp_flag); fr(c->gp_Xs_f); fr(c->gp_T);
  fr(c->gp_LinvT); fr(c->gp_LinvT_f); fr(c->gp_ctr); fr(c->gp_XsT); fr(c->ucand.p);
  fr(c->gp_XsT_num.p); fr(c->gp_xnorm_num.p); fr(c->gp_acat.p); fr(c->bcat.p); fr(c->pr_bcat.p);
  fr(c->gp_i8a.p); fr(c->gp_i8rs.p);
  fr(c->gp_x8.p); fr(c->u8.p); fr(c->gp_q8.p); fr(c->scol.p);
  fr(c->kst.p); fr(c->mu_part.p); fr(c->var_part.p); fr(c->cnorm.p);
  fr(c->r_values.p); fr(c->r_feat.p); fr(c->r_mu.p); fr(c->r_var.p); fr(c->r_score.p); fr(c->r_digest.p);
  fr(c->r_dup.p); fr(c->tk_score[0].p); fr(c->tk_score[1].p); fr(c->tk_idx[0].p); fr(c->tk_idx[1].p);
  fr(c->r_topk_idx.p); fr(c->r_topk_score.p); fr(c->perm_ws.p); fr(c->perm_dig.p);
  fr(c->forest_nodes); fr(c->forest_roots); fr(c->r_topk_vals.p);
  fr(c->cm_send.p); fr(c->cm_recv.p); fr(c->cm_keep.p); fr(c->cm_pay.p); fr(c->cm_cnt.p);
  for (auto& m : c->timing.marks) hipEventDestroy(m.ev);
  for (hipEvent_t e : {c->ev_fork, c->ev_join, c->ev_fit, c->ev_prefit, c->ev_fit_x})
    if (e) hipEventDestroy(e);
  if (c->fit_host) hipHostFree(c->fit_host);
  if (c->flag_host) hipHostFree(c->flag_host);
  for (hipStream_t st : {c->own_stream, c->side, c->fit_stream})
    if (st) hipStreamDestroy(st);
  delete c;
  return 0;
}

const char* ut_last_error(ut_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ut_set_stream(ut_ctx* c, void* s) {
  if (!c) return UT_EINVAL;
  if (int rc = gp_fit_flush(c)) return rc;   // (ordered on the stream it was staged against)
  c->stream = (hipStream_t)s;  // NULL = the device's default (null) stream
  return 0;
}

int ut_sync(ut_ctx* c) {
  if (!c) return UT_EINVAL;
  if (int rc = gp_fit_flush(c)) return rc;
  UT_HIP(c, ut::sync_all(c));
  return 0;
}

int ut_space_define(ut_ctx* c, int32_t P, const ut_param_desc* params, int32_t py2_layout) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, P >= 1 && params, UT_EINVAL, "space: need at least one parameter");
  UT_HIP(c, hipSetDevice(c->device));
  if (int rc = gp_fit_flush(c)) return rc;   // a staged fit reads the space's categorical layout
  UT_HIP(c, ut::sync_all(c));
  free_space(c->space);
  c->has_space = false;
  Space& s = c->space;
  s.P = P;
  s.py2 = py2_layout ? 1 : 0;
  s.host_params.resize(P);
  s.host_order.assign(P, -1);
  std::vector<std::string> names(P);
  std::vector<bool> primitive(P);
  std::vector<uint32_t> lut;
  std::vector<double> vtab;
  std::vector<int32_t> perm_params, perm_off, perm_offbase, perm_len, comp;
  std::vector<uint8_t> perm_bytes;
  int32_t feat = 0, col = 0;
  for (int32_t p = 0; p < P; ++p) {
    const ut_param_desc& d = params[p];
    DevParam& q = s.host_params[p];
    q.kind = d.kind;
    q.col = col;
    q.psize = 1;
    q.wcol = 0;
    q.pslot = -1;
    q.cslot = -1;
    q.pad_ = 0;
    q.lo = d.lo; q.hi = d.hi;
    q.u_lo = d.u_lo; q.u_hi = d.u_hi; q.u_span = d.u_span;
    q.n_opt = d.n_options;
    q.feat_col = feat;
    q.vtab_base = 0;
    q.vtab_n = 0;
    UT_CHECK(c, d.sort_rank >= 0 && d.sort_rank < P && s.host_order[d.sort_rank] == -1, UT_EINVAL,
             "space: sort_rank must be a permutation of 0..P-1");
    s.host_order[d.sort_rank] = p;
    names[p] = std::string(d.name ? d.name : "", d.name ? (size_t)d.name_len : 0);
    switch (d.kind) {
      case UT_FLOAT: case UT_INT: case UT_LOGINT:
        q.n_feat = 1; primitive[p] = true; break;
      case UT_POW2: {
        // searched by exponent: legal_range = (log2 min, log2 max)  (manipulator.py:829-830)
        UT_CHECK(c, d.lo >= 1.0 && d.hi >= d.lo && d.hi <= 0x1p1023, UT_EINVAL, "space: bad PowerOfTwo range");
        int elo = 0, ehi = 0;
        UT_CHECK(c, frexp(d.lo, &elo) == 0.5 && frexp(d.hi, &ehi) == 0.5, UT_EINVAL,
                 "space: PowerOfTwo bounds must be powers of two");
        q.lo = (double)(elo - 1);
        q.hi = (double)(ehi - 1);
        q.n_feat = 1; primitive[p] = true; break;
      }
      case UT_BOOL:
        q.n_feat = 1; primitive[p] = false; q.n_opt = 2; break;
      case UT_ENUM:
        UT_CHECK(c, d.n_options >= 1, UT_EINVAL, "space: enum needs options");
        q.n_feat = (int32_t)d.n_options; primitive[p] = false; break;
      case UT_PERM: {
        // PermutationParameter(name, items): S columns of item indices,
        // inner digest sha256(repr(list)) computed on the device from the
        // items' repr bytes (a fixed-length message per space)
        UT_CHECK(c, d.n_options >= 1 && d.n_options <= 65536, UT_EINVAL, "space: permutation size must be in [1, 65536]");
        UT_CHECK(c, d.perm_repr_host && d.perm_repr_off_host, UT_EINVAL, "space: permutation needs item reprs");
        const int32_t S = (int32_t)d.n_options;
        q.psize = S;
        q.n_opt = S;
        q.n_feat = S;
        q.wcol = s.perm_cols;
        q.pslot = s.n_perm;
        q.hash_mode = HM_PERM;
        primitive[p] = false;
        perm_params.push_back(p);
        perm_offbase.push_back((int32_t)perm_off.size());
        const int32_t base = (int32_t)perm_bytes.size();
        const int32_t* off = d.perm_repr_off_host;
        UT_CHECK(c, off[0] == 0, UT_EINVAL, "space: permutation repr offsets must start at 0");
        for (int32_t k = 0; k < S; ++k)
          UT_CHECK(c, off[k + 1] > off[k], UT_EINVAL, "space: empty item repr");
        perm_bytes.insert(perm_bytes.end(), d.perm_repr_host, d.perm_repr_host + off[S]);
        for (int32_t k = 0; k <= S; ++k) perm_off.push_back(base + off[k]);
        perm_len.push_back(2 + off[S] + 2 * (S - 1));  // "[" items joined by ", " "]"
        s.n_perm += 1;
        s.perm_cols += S;
        if (S > s.perm_smax) s.perm_smax = S;
        break;
      }
      default:
        return set_err(c, UT_EUNSUPPORTED, "space: parameter kind " + std::to_string(d.kind) +
                                               " is not supported on the device path yet");
    }
    feat += q.n_feat;
    col += q.psize;
    if (d.kind == UT_PERM) continue;
    if (d.kind == UT_LOGINT && d.vtab_count > 0) {
      UT_CHECK(c, d.vtab_host != nullptr, UT_EINVAL, "space: vtab_count > 0 but vtab_host is NULL");
      q.vtab_base = (int64_t)vtab.size();
      q.vtab_n = d.vtab_count;
      vtab.insert(vtab.end(), d.vtab_host, d.vtab_host + d.vtab_count);
    }
    if (d.lut_count > 0) {
      UT_CHECK(c, d.lut_host != nullptr, UT_EINVAL, "space: lut_count > 0 but lut_host is NULL");
      q.hash_mode = HM_LUT;
      q.lut_base = (int64_t)(lut.size() / 8);
      q.lut_n = d.lut_count;
      for (int32_t v = 0; v < d.lut_count; ++v)
        for (int w = 0; w < 8; ++w) {
          const uint8_t* b = d.lut_host + (size_t)v * 32 + 4 * w;
          lut.push_back(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]);
        }
    } else {
      q.lut_base = 0;
      q.lut_n = 0;
      if (d.kind == UT_FLOAT) q.hash_mode = HM_FLOAT;
      else if (d.kind == UT_INT) q.hash_mode = HM_INT;
      else if (d.kind == UT_LOGINT) q.hash_mode = HM_LOGINT;
      else return set_err(c, UT_EINVAL, "space: BOOL/ENUM/POW2 parameters need an inner-digest LUT");
      q.cslot = s.n_comp++;
      comp.push_back(p);
    }
  }
  s.n_feat = feat;
  s.ncols = col;
  UT_HIP(c, ut::dmalloc((void**)&s.d_params, sizeof(DevParam) * P));
  UT_HIP(c, hipMemcpy(s.d_params, s.host_params.data(), sizeof(DevParam) * P, hipMemcpyHostToDevice));
  UT_HIP(c, ut::dmalloc((void**)&s.d_order, sizeof(int32_t) * P));
  UT_HIP(c, hipMemcpy(s.d_order, s.host_order.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice));
  if (lut.empty()) lut.resize(8, 0u);
  {  // the device LUT holds each digest as its 64 hex characters (16 big-endian
     // words, what the outer message holds): k_hash copies them into its hex slot
    std::vector<uint32_t> luthex(lut.size() * 2);
    for (size_t e = 0; e < lut.size() / 8; ++e) ut::digest_hex(&lut[8 * e], &luthex[16 * e]);
    UT_HIP(c, ut::dmalloc((void**)&s.d_lut, sizeof(uint32_t) * luthex.size()));
    UT_HIP(c, hipMemcpy(s.d_lut, luthex.data(), sizeof(uint32_t) * luthex.size(), hipMemcpyHostToDevice));
  }
  if (vtab.empty()) vtab.resize(1, 0.0);
  UT_HIP(c, ut::dmalloc((void**)&s.d_vtab, sizeof(double) * vtab.size()));
  UT_HIP(c, hipMemcpy(s.d_vtab, vtab.data(), sizeof(double) * vtab.size(), hipMemcpyHostToDevice));
  {
    std::vector<int32_t> order_col(P);
    for (int32_t j = 0; j < P; ++j) order_col[j] = s.host_params[s.host_order[j]].col;
    UT_HIP(c, ut::dmalloc((void**)&s.d_order_col, sizeof(int32_t) * P));
    UT_HIP(c, hipMemcpy(s.d_order_col, order_col.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice));
  }
  if (s.n_perm > 0) {
    auto up = [&](auto*& dst, const auto& v) -> hipError_t {
      hipError_t e = ut::dmalloc((void**)&dst, sizeof(v[0]) * v.size());
      if (e != hipSuccess) return e;
      return hipMemcpy(dst, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice);
    };
    UT_HIP(c, up(s.d_perm_params, perm_params));
    UT_HIP(c, up(s.d_perm_bytes, perm_bytes));
    UT_HIP(c, up(s.d_perm_off, perm_off));
    UT_HIP(c, up(s.d_perm_offbase, perm_offbase));
    UT_HIP(c, up(s.d_perm_len, perm_len));
  }
  if (s.n_comp > 0) {
    UT_HIP(c, ut::dmalloc((void**)&s.d_comp, sizeof(int32_t) * comp.size()));
    UT_HIP(c, hipMemcpy(s.d_comp, comp.data(), sizeof(int32_t) * comp.size(), hipMemcpyHostToDevice));
  }
  {
    std::vector<int32_t> col_param(s.ncols > 0 ? s.ncols : 1, -1);
    for (int32_t j = 0; j < P; ++j)
      if (s.host_params[j].kind != UT_PERM) col_param[s.host_params[j].col] = j;
    UT_HIP(c, ut::dmalloc((void**)&s.d_col_param, sizeof(int32_t) * col_param.size()));
    UT_HIP(c, hipMemcpy(s.d_col_param, col_param.data(), sizeof(int32_t) * col_param.size(), hipMemcpyHostToDevice));
  }
  {  // categorical K*: ENUM / BOOL code columns, numeric features (gp_gemm.hip)
    std::vector<int32_t> ccol(P, -1), feat_num(s.n_feat > 0 ? s.n_feat : 1, -1);
    int32_t kc = 0;
    for (int32_t p = 0; p < P; ++p) {
      const DevParam& q = s.host_params[p];
      if (q.kind == UT_ENUM || q.kind == UT_BOOL) {
        ccol[p] = kc;
        kc += q.kind == UT_ENUM ? (int32_t)q.n_opt : 2;
        s.host_cat.push_back(p);
      } else {
        for (int32_t f = 0; f < q.n_feat; ++f) {
          feat_num[q.feat_col + f] = (int32_t)s.host_num_feat.size();
          s.host_num_feat.push_back(q.feat_col + f);
        }
      }
    }
    s.n_cat = (int32_t)s.host_cat.size();
    s.n_num = (int32_t)s.host_num_feat.size();
    s.cat_k = (kc + 127) / 128 * 128;
    std::vector<int32_t> num_feat = s.host_num_feat;
    if (num_feat.empty()) num_feat.push_back(0);
    UT_HIP(c, ut::dmalloc((void**)&s.d_cat_ccol, sizeof(int32_t) * P));
    UT_HIP(c, hipMemcpy(s.d_cat_ccol, ccol.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice));
    UT_HIP(c, ut::dmalloc((void**)&s.d_num_feat, sizeof(int32_t) * num_feat.size()));
    UT_HIP(c, hipMemcpy(s.d_num_feat, num_feat.data(), sizeof(int32_t) * num_feat.size(), hipMemcpyHostToDevice));
    UT_HIP(c, ut::dmalloc((void**)&s.d_feat_num, sizeof(int32_t) * feat_num.size()));
    UT_HIP(c, hipMemcpy(s.d_feat_num, feat_num.data(), sizeof(int32_t) * feat_num.size(), hipMemcpyHostToDevice));
  }
  int rc = compile_hash_layout(c, names, primitive);
  if (rc) return rc;
  c->has_space = true;
  // a new space invalidates the population (and its digest cache)
  if (c->pop) {
    ut::dfree(c->pop);
    c->pop = nullptr;
    c->npop = 0;
    c->pop_cap = 0;
  }
  c->pop_dig_valid = false;
  c->pop_aos_valid = false;
  for (auto& ps : c->pop_slots) ps.pop_dig_valid = ps.pop_aos_valid = false;
  return 0;
}

int ut_space_info(ut_ctx* c, int64_t* outer_len, int64_t* outer_blocks, int32_t* n_features) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  if (outer_len) *outer_len = c->space.outer_len;
  if (outer_blocks) *outer_blocks = c->space.outer_blocks;
  if (n_features) *n_features = c->space.n_feat;
  return 0;
}

int ut_space_columns(ut_ctx* c, int32_t* n_columns) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  if (n_columns) *n_columns = c->space.ncols;
  return 0;
}

static int pop_alloc(ut_ctx* c, int64_t npop) {
  const int64_t need = npop * c->space.ncols;
  if (c->pop && c->pop_cap >= need) {
    c->npop = npop;
    return 0;
  }
  if (c->pop) {
    UT_HIP(c, ut::sync_all(c));
    ut::dfree(c->pop);
  }
  UT_HIP(c, ut::dmalloc((void**)&c->pop, sizeof(double) * need));
  c->pop_cap = need;
  c->npop = npop;
  return 0;
}

int ut_population_init(ut_ctx* c, int64_t npop, uint32_t round_) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, npop >= 4 && npop < (int64_t)0xFFFFFFFF, UT_EINVAL, "population size must be in [4, 2^32)");
  int rc = pop_alloc(c, npop);
  if (rc) return rc;
  c->pop_dig_valid = false;
  c->pop_aos_valid = false;
  return launch_population_init(c, round_);
}

int ut_population_set(ut_ctx* c, int64_t npop, const double* values, int64_t ld) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, npop >= 4 && npop < (int64_t)0xFFFFFFFF && values && ld >= npop, UT_EINVAL,
           "population_set: bad arguments");
  int rc = pop_alloc(c, npop);
  if (rc) return rc;
  c->pop_dig_valid = false;
  c->pop_aos_valid = false;
  UT_HIP(c, hipMemcpy2DAsync(c->pop, sizeof(double) * npop, values, sizeof(double) * ld, sizeof(double) * npop,
                             c->space.ncols, hipMemcpyDeviceToDevice, c->stream));
  return 0;
}

int ut_population_select(ut_ctx* c, int32_t slot) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, slot >= 0 && slot < 1024, UT_EINVAL, "population_select: slot must be in [0, 1024)");
  if (slot == c->pop_slot) return 0;
  if ((int32_t)c->pop_slots.size() <= std::max(slot, c->pop_slot))
    c->pop_slots.resize(std::max(slot, c->pop_slot) + 1);
  // park the current slot, load the requested one (host-side pointer swap:
  // launches already enqueued keep the pointers they were given)
  ut_ctx::PopSlot& cur = c->pop_slots[c->pop_slot];
  cur.pop = c->pop; cur.npop = c->npop; cur.pop_cap = c->pop_cap;
  cur.pso_vel = c->pso_vel; cur.pso_best = c->pso_best; cur.pso_cap = c->pso_cap;
  cur.pop_dig = c->pop_dig; cur.pop_dig_cap = c->pop_dig_cap; cur.pop_dig_valid = c->pop_dig_valid;
  cur.pop_dig_lo = c->pop_dig_lo; cur.pop_dig_n = c->pop_dig_n;
  cur.pop_aos = c->pop_aos; cur.pop_aos_cap = c->pop_aos_cap; cur.pop_aos_valid = c->pop_aos_valid;
  const ut_ctx::PopSlot& nx = c->pop_slots[slot];
  c->pop = nx.pop; c->npop = nx.npop; c->pop_cap = nx.pop_cap;
  c->pso_vel = nx.pso_vel; c->pso_best = nx.pso_best; c->pso_cap = nx.pso_cap;
  c->pop_dig = nx.pop_dig; c->pop_dig_cap = nx.pop_dig_cap; c->pop_dig_valid = nx.pop_dig_valid;
  c->pop_dig_lo = nx.pop_dig_lo; c->pop_dig_n = nx.pop_dig_n;
  c->pop_aos = nx.pop_aos; c->pop_aos_cap = nx.pop_aos_cap; c->pop_aos_valid = nx.pop_aos_valid;
  c->pop_slot = slot;
  return 0;
}

int ut_population_get(ut_ctx* c, double* values, int64_t ld) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->pop != nullptr && values && ld >= c->npop, UT_EINVAL, "population_get: bad arguments");
  UT_HIP(c, hipMemcpy2DAsync(values, sizeof(double) * ld, c->pop, sizeof(double) * c->npop,
                             sizeof(double) * c->npop, c->space.ncols, hipMemcpyDeviceToDevice, c->stream));
  return 0;
}

static int check_de_params(ut_ctx* c, const ut_de_params* p, int64_t m, int64_t cand_base) {
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, c->pop != nullptr, UT_EINVAL, "propose_de: population not initialised");
  UT_CHECK(c, p && p->n_cross >= 0 && p->n_cross <= 4, UT_EINVAL, "propose_de: n_cross must be in [0, 4]");
  UT_CHECK(c, p->information_sharing >= 0 && p->information_sharing <= (1 << 20), UT_EINVAL,
           "propose_de: information_sharing must be in [0, 2^20]");
  UT_CHECK(c, c->npop - 1 + (p->best ? (int64_t)p->information_sharing : 0) >= 3, UT_EINVAL,
           "propose_de: the donor pool (population - target + best copies) needs >= 3 entries");
  UT_CHECK(c, m >= 0 && cand_base >= 0, UT_EINVAL, "propose_de: bad arguments");
  return 0;
}

int ut_propose_de(ut_ctx* c, const ut_de_params* p, uint32_t round_, int64_t cand_base, int64_t m,
                  double* out_values, int64_t ld) {
  if (!c) return UT_EINVAL;
  int rc = check_de_params(c, p, m, cand_base);
  if (rc) return rc;
  UT_CHECK(c, (out_values || m == 0) && ld >= m, UT_EINVAL, "propose_de: bad arguments");
  if (m == 0) return 0;
  // a staged fit is issued after the proposal (as in score_round_de_impl)
  if ((rc = gp_fit_prefit(c))) return rc;
  if ((rc = launch_de(c, p, round_, cand_base, m, out_values, ld))) return rc;
  return gp_fit_flush(c);
}

int ut_encode_features(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* feat, int64_t ldf) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, m >= 0 && ((values && feat) || m == 0) && ld >= m && ldf >= m, UT_EINVAL, "encode: bad arguments");
  if (m == 0) return 0;
  return launch_encode(c, values, ld, m, feat, ldf);
}

int ut_hash(ut_ctx* c, const double* values, int64_t ld, int64_t m, uint32_t* out) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, m >= 0 && ((values && out) || m == 0) && ld >= m, UT_EINVAL, "hash: bad arguments");
  return launch_hash(c, values, ld, m, out);
}

int ut_hash_de(ut_ctx* c, const double* values, int64_t ld, int64_t m, int64_t cand_base, uint32_t* out) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, c->pop != nullptr, UT_EINVAL, "hash_de: population not initialised");
  UT_CHECK(c, m >= 0 && cand_base >= 0 && ((values && out) || m == 0) && ld >= m, UT_EINVAL, "hash_de: bad arguments");
  return launch_hash_de(c, values, ld, m, cand_base, out);
}

int ut_hash_parent(ut_ctx* c, const double* values, int64_t ld, int64_t m, const double* parent, uint32_t* out) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, m >= 0 && parent && ((values && out) || m == 0) && ld >= m, UT_EINVAL, "hash_parent: bad arguments");
  return launch_hash_parent(c, values, ld, m, parent, out);
}

int ut_history_reset(ut_ctx* c, int64_t capacity) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, capacity >= 0, UT_EINVAL, "history capacity < 0");
  return history_alloc(c, capacity * 2 > 1024 ? capacity * 2 : 1024);
}

int ut_history_add(ut_ctx* c, const uint32_t* dig, int64_t n) {
  if (!c) return UT_EINVAL;
  if (n <= 0) return 0;
  UT_CHECK(c, dig != nullptr, UT_EINVAL, "history_add: NULL digests");
  if (!c->hist_keys || (c->hist_count + n) * 2 > c->hist_cap) {
    // grow: rebuild is not needed for correctness of membership if we keep
    // the old entries, so re-insert by copying old keys
    const int64_t old_cap = c->hist_cap;
    uint32_t* old_keys = c->hist_keys;
    uint32_t* old_state = c->hist_state;
    const int64_t old_count = c->hist_count;
    c->hist_keys = nullptr;
    c->hist_state = nullptr;
    int64_t want = (old_count + n) * 4;
    int64_t p2 = 1024;
    while (p2 < want) p2 <<= 1;
    UT_HIP(c, ut::dmalloc((void**)&c->hist_keys, sizeof(uint32_t) * 8 * p2));
    UT_HIP(c, ut::dmalloc((void**)&c->hist_state, sizeof(uint32_t) * p2));
    UT_HIP(c, hipMemsetAsync(c->hist_state, 0, sizeof(uint32_t) * p2, c->stream));
    c->hist_cap = p2;
    c->hist_count = 0;
    if (old_keys) {
      int rc = launch_hist_rehash(c, old_keys, old_state, old_cap);
      UT_HIP(c, ut::sync_all(c));
      ut::dfree(old_keys);
      ut::dfree(old_state);
      if (rc) return rc;
      c->hist_count = old_count;
    }
  }
  int rc = launch_hist_insert(c, dig, n);
  if (rc) return rc;
  c->hist_count += n;
  return 0;
}

int ut_history_add_host(ut_ctx* c, const uint32_t* dig, int64_t n) {
  if (!c) return UT_EINVAL;
  if (n <= 0) return 0;
  UT_CHECK(c, dig != nullptr, UT_EINVAL, "history_add_host: NULL digests");
  uint32_t* tmp = nullptr;
  UT_HIP(c, ut::dmalloc((void**)&tmp, sizeof(uint32_t) * 8 * n));
  UT_HIP(c, hipMemcpyAsync(tmp, dig, sizeof(uint32_t) * 8 * n, hipMemcpyHostToDevice, c->stream));
  int rc = ut_history_add(c, tmp, n);
  UT_HIP(c, ut::sync_all(c));
  ut::dfree(tmp);
  return rc;
}

int ut_dedup(ut_ctx* c, const uint32_t* dig, int64_t m, uint8_t* dup) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, m >= 0 && ((dig && dup) || m == 0), UT_EINVAL, "dedup: bad arguments");
  return launch_dedup(c, dig, m, dup);
}

int ut_gp_fit(ut_ctx* c, const double* X, const double* y, int32_t n, int32_t d, const ut_gp_hyper* h) {
  if (!c) return UT_EINVAL;
  UT_HIP(c, hipSetDevice(c->device));
  int rc = gp_fit_enqueue(c, X, y, n, d, h);
  if (rc) return rc;
  return gp_wait_fit(c);
}

int ut_gp_fit_async(ut_ctx* c, const double* X, const double* y, int32_t n, int32_t d, const ut_gp_hyper* h) {
  if (!c) return UT_EINVAL;
  UT_HIP(c, hipSetDevice(c->device));
  return gp_fit_enqueue(c, X, y, n, d, h);
}

int ut_gp_join_fit(ut_ctx* c) {
  if (!c) return UT_EINVAL;
  if (int rc = gp_fit_flush(c)) return rc;
  if (c->fit_pending) UT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_fit, 0));
  return 0;
}

int ut_gp_set_fit_append(ut_ctx* c, int32_t enable) {
  if (!c) return UT_EINVAL;
  c->fit_append = enable != 0;
  return 0;
}

int ut_gp_last_fit_kind(ut_ctx* c, int32_t* kind) {
  if (!c || !kind) return UT_EINVAL;
  *kind = c->gp_fit_kind;
  return 0;
}

int ut_gp_score(ut_ctx* c, const double* feat, int64_t ld, int64_t m, const ut_acq* acq, const uint8_t* dup,
                double* mu, double* var, double* score) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, m >= 0 && (feat || m == 0) && ld >= m, UT_EINVAL, "gp_score: bad arguments");
  // a stand-alone scoring call is a timing round of its own (stages kstar, var, finalize)
  const bool own = c->timing.on && !c->timing.in_round;
  if (own) timing_begin(c);
  int rc = gp_score_impl(c, feat, ld, m, acq, dup, mu, var, score);
  if (own) timing_end(c);
  return rc;
}

int ut_gp_score_values(ut_ctx* c, const double* values, int64_t ld, int64_t m, const ut_acq* acq,
                       const uint8_t* dup, double* mu, double* var, double* score) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, m >= 0 && (values || m == 0) && ld >= m, UT_EINVAL, "gp_score_values: bad arguments");
  UT_CHECK(c, acq != nullptr, UT_EINVAL, "gp_score: acq is NULL");
  const bool own = c->timing.on && !c->timing.in_round;
  if (own) timing_begin(c);
  // encode + 1/ell scaling + |u'|^2 in one pass (k_encode_scaled): no feature matrix
  int rc = gp_encode_scaled(c, values, ld, m);
  mark(c, "encode");   // (else the encode's time would land in the next stage, fit_wait)
  if (!rc) rc = gp_score_impl(c, nullptr, ld, m, acq, dup, mu, var, score);
  if (own) timing_end(c);
  return rc;
}

int ut_gp_topk_pruned(ut_ctx* c, const double* feat, int64_t ld, int64_t m, const ut_acq* acq, const uint8_t* dup,
                      int64_t cand_base, int32_t k, int32_t bound_rows, int64_t* out_idx, double* out_score,
                      ut_prune_stats* stats) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, m >= 1 && feat && ld >= m && acq && out_idx && out_score && cand_base >= 0, UT_EINVAL,
           "gp_topk_pruned: bad arguments");
  const bool own = c->timing.on && !c->timing.in_round;
  if (own) timing_begin(c);
  int rc = gp_topk_pruned_impl(c, feat, ld, m, acq, dup, cand_base, k, bound_rows, out_idx, out_score, stats);
  if (own) timing_end(c);
  return rc;
}

int ut_gp_set_precision(ut_ctx* c, int32_t bits) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, bits == 64 || bits == 32 || bits == 16 || bits == 8, UT_EINVAL,
           "gp precision must be 64, 32, 16 (f16x3) or 8 (int8 slices, fp64 tier)");
  if (int rc = gp_fit_flush(c)) return rc;   // a staged fit was sized for the precision it was staged at
  c->gp_prec = bits;
  return 0;
}

int ut_gp_set_prune_pass(ut_ctx* c, int32_t bits) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, bits == 32 || bits == 64, UT_EINVAL, "prune pass must be 32 or 64");
  c->prune_pass = bits;
  return 0;
}

int ut_gp_set_i8_tol(ut_ctx* c, double tol) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, tol >= 0.0 && tol < 1.0, UT_EINVAL, "i8 tolerance must be in [0, 1)");
  c->i8_tol = tol;
  return 0;
}

int ut_gp_i8_bounds(ut_ctx* c, double* E, double* Emu) {
  if (!c) return UT_EINVAL;
  if (int rc = gp_fit_flush(c)) return rc;
  double b[2] = {0.0, 0.0};
  if (c->gp_fit_prec == 8 && c->gp_i8rs.p) {
    UT_HIP(c, hipStreamSynchronize(c->fit_stream));
    UT_HIP(c, hipMemcpy(b, c->gp_i8rs.p + 2 * (int64_t)c->gp_npad_fit, sizeof(b), hipMemcpyDeviceToHost));
  }
  if (E) *E = b[0];
  if (Emu) *Emu = b[1];
  return 0;
}

int ut_gp_i8_stats(ut_ctx* c, int64_t* recomputed, double* bound) {
  if (!c) return UT_EINVAL;
  if (int rc = gp_fit_flush(c)) return rc;
  if (recomputed) *recomputed = c->i8_recomputed;
  if (bound) {
    *bound = 0.0;
    if (c->gp_fit_prec == 8 && c->gp_i8rs.p) {
      UT_HIP(c, hipStreamSynchronize(c->fit_stream));
      UT_HIP(c, hipMemcpy(bound, c->gp_i8rs.p + 2 * (int64_t)c->gp_npad_fit, sizeof(double), hipMemcpyDeviceToHost));
    }
  }
  return 0;
}

int ut_gp_fit_status(ut_ctx* c, int32_t* ok) {
  if (!c || !ok) return UT_EINVAL;
  UT_CHECK(c, c->gp_ready || c->fit_pending, UT_EINVAL, "gp_fit_status: no fit");
  const int rc = gp_wait_fit(c);
  if (rc != 0 && rc != UT_ENOTPD) return rc;
  *ok = rc == 0 ? 1 : 0;
  return 0;
}

int ut_gp_kstar_mode(ut_ctx* c, int32_t* categorical) {
  if (!c || !categorical) return UT_EINVAL;
  *categorical = c->cat_on ? 1 : 0;
  return 0;
}

int ut_gp_stats(ut_ctx* c, double* f_best, double* y_mean, double* y_std) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->gp_ready, UT_EINVAL, "gp_stats: no fitted GP");
  int rc = gp_wait_fit(c);
  if (rc) return rc;
  double st[4];
  UT_HIP(c, hipMemcpyAsync(st, c->gp_stats, sizeof(double) * 3, hipMemcpyDeviceToHost, c->stream));
  UT_HIP(c, ut::sync_all(c));
  if (f_best) *f_best = st[0];
  if (y_mean) *y_mean = st[1];
  if (y_std) *y_std = st[2];
  return 0;
}

int ut_topk(ut_ctx* c, const double* score, const uint8_t* dup, int64_t m, int64_t cand_base, int32_t k,
            int64_t* out_idx, double* out_score) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, score || m == 0, UT_EINVAL, "topk: NULL score");
  return topk_impl(c, score, dup, m, cand_base, k, out_idx, out_score);
}

static int round_outputs(ut_ctx* c, const ut_round_out* out, int64_t ld, int64_t cand_base, int32_t k);
static int score_round_de_impl(ut_ctx* c, const ut_de_params* de, const ut_acq* acq, uint32_t round_,
                               int64_t cand_base, int64_t m, int32_t k, const ut_round_out* out, int32_t prune_rows,
                               ut_prune_stats* stats);

int ut_score_round_de(ut_ctx* c, const ut_de_params* de, const ut_acq* acq, uint32_t round_, int64_t cand_base,
                      int64_t m, int32_t k, const ut_round_out* out) {
  return score_round_de_impl(c, de, acq, round_, cand_base, m, k, out, 0, nullptr);
}

int ut_score_round_de_pruned(ut_ctx* c, const ut_de_params* de, const ut_acq* acq, uint32_t round_,
                             int64_t cand_base, int64_t m, int32_t k, int32_t bound_rows, const ut_round_out* out,
                             ut_prune_stats* stats) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, bound_rows >= 1, UT_EINVAL, "score_round_pruned: bound_rows must be >= 1");
  return score_round_de_impl(c, de, acq, round_, cand_base, m, k, out, bound_rows, stats);
}

static int score_round_de_impl(ut_ctx* c, const ut_de_params* de, const ut_acq* acq, uint32_t round_,
                               int64_t cand_base, int64_t m, int32_t k, const ut_round_out* out, int32_t prune_rows,
                               ut_prune_stats* stats) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, c->pop != nullptr, UT_EINVAL, "score_round: population not initialised");
  UT_CHECK(c, c->gp_ready, UT_EINVAL, "score_round: call ut_gp_fit first");
  UT_CHECK(c, c->gp_d == c->space.n_feat, UT_EINVAL, "score_round: GP feature width != space feature width");
  UT_CHECK(c, m >= 1 && de && acq, UT_EINVAL, "score_round: bad arguments");
  const int64_t ld = ((m + 127) / 128) * 128;
  const int32_t NC = c->space.ncols;
  int rc;
  if ((rc = ensure(c, c->r_values, (size_t)NC * ld))) return rc;
  if ((rc = ensure(c, c->r_digest, (size_t)8 * ld))) return rc;
  if ((rc = ensure(c, c->r_dup, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_mu, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_var, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_score, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_topk_idx, (size_t)k))) return rc;
  if ((rc = ensure(c, c->r_topk_score, (size_t)k))) return rc;
  c->r_ld = ld;
  c->r_m = m;
  timing_begin(c);
  // the proposal also writes the DE-diff mask / pairs the hash reuses
  if ((rc = check_de_params(c, de, m, cand_base))) return rc;
  // a staged fit (ut_gp_fit_async) keeps its place before the proposal but is
  // issued after it: the proposal runs while the host issues the fit
  if ((rc = gp_fit_prefit(c))) return rc;
  if ((rc = launch_de(c, de, round_, cand_base, m, c->r_values.p, ld, true))) return rc;
  if ((rc = gp_fit_flush(c))) return rc;
  mark(c, "propose");
  // fork: hash_config + dedup on the side stream, beside encode + GP scoring.
  // Dense fp64 rounds (the only ones whose K* does not wait for the whole
  // fit) hold the hash for an in-flight fit: beside the full hash grid the
  // fit's chain of small kernels stretches from ~1.5 to ~9 ms and the
  // variance GEMM waits for it; held, the fit runs beside K* alone (C2:
  // 26.10 ms per round, against 26.32 holding only the outer hash and 26.54
  // holding nothing; round 3).
  auto fork_hash = [&]() -> int {
    UT_HIP(c, hipEventRecord(c->ev_fork, c->stream));
    UT_HIP(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
    StreamScope on_side(c, c->side);
    mark(c, "");
    c->round_hash_hold = prune_rows == 0 && c->gp_fit_prec == 64;
    int r = launch_hash_de(c, c->r_values.p, ld, m, cand_base, c->r_digest.p, true);
    c->round_hash_hold = false;
    if (r) return r;
    mark(c, "hash");
    if ((r = launch_dedup(c, c->r_digest.p, m, c->r_dup.p))) return r;
    mark(c, "dedup");
    UT_HIP(c, hipEventRecord(c->ev_join, c->side));
    return 0;
  };
  if ((rc = fork_hash())) return rc;
  // encode straight into the K* operands (features * 1/ell, their norms and
  // the one-hot codes); the pruned round gathers its threshold set's and
  // survivors' columns from those (C3 pruned: encode 1.07 + prep 2.1 ms ->
  // one fused pass)
  if ((rc = gp_encode_scaled(c, c->r_values.p, ld, m))) return rc;
  c->r_feat_valid = false;
  mark(c, "encode");
  if (prune_rows > 0) {
    // pruned: only candidates whose score bound reaches the threshold get the
    // full variance (the bound kernel joins the dup mask first)
    if ((rc = gp_topk_pruned_impl(c, nullptr, ld, m, acq, c->r_dup.p, cand_base, k, prune_rows, c->r_topk_idx.p,
                                  c->r_topk_score.p, stats, c->ev_join, true)))
      return rc;
  } else {
    // the variance GEMM joins the side stream's hash + dedup (they share the
    // CUs with K* only), the finalize kernel masks duplicates
    if ((rc = gp_score_impl(c, nullptr, ld, m, acq, c->r_dup.p, c->r_mu.p, c->r_var.p, c->r_score.p, c->ev_join)))
      return rc;
    if ((rc = topk_impl(c, c->r_score.p, c->r_dup.p, m, cand_base, k, c->r_topk_idx.p, c->r_topk_score.p)))
      return rc;
    mark(c, "topk");
  }
  if ((rc = round_outputs(c, out, ld, cand_base, k))) return rc;
  mark(c, "outputs");
  return timing_end(c);
}

// a round's selections to the caller: indices, scores, rows and digests
static int round_outputs(ut_ctx* c, const ut_round_out* out, int64_t ld, int64_t cand_base, int32_t k) {
  if (!out) return 0;
  int rc;
  if (out->topk_idx)
    UT_HIP(c, hipMemcpyAsync(out->topk_idx, c->r_topk_idx.p, sizeof(int64_t) * k, hipMemcpyDeviceToDevice,
                             c->stream));
  if (out->topk_score)
    UT_HIP(c, hipMemcpyAsync(out->topk_score, c->r_topk_score.p, sizeof(double) * k, hipMemcpyDeviceToDevice,
                             c->stream));
  if (out->topk_values || out->topk_digest) {
    double* vals = out->topk_values;
    if (!vals) {  // digests only: the rows go to a context buffer (no per-round alloc / sync)
      if ((rc = ensure(c, c->r_topk_vals, (size_t)c->space.ncols * k))) return rc;
      vals = c->r_topk_vals.p;
    }
    if ((rc = launch_gather_rows(c, c->r_values.p, ld, c->r_topk_idx.p, cand_base, k, vals, k, c->r_digest.p,
                                 out->topk_digest)))
      return rc;
  }
  return 0;
}

// A GA / GGA scoring round (ut_score_round_ga): the children of parent1
// (evolutionarytechniques.py:29-61, globalGA.py:28-48 and :68-76), then hash_config of
// the children (the parent's inner digests reused) + dedup on the side stream
// beside the fused encode and the GP scoring, their invalid children joined to
// the duplicates, top-k.  What the C4 round ran as separate calls on one stream.
int ut_score_round_ga(ut_ctx* c, const ut_ga_params* ga, const double* parent1, const double* parent2,
                      const ut_acq* acq, uint32_t round_, int64_t cand_base, int64_t m, int32_t k,
                      const ut_round_out* out) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, c->gp_ready, UT_EINVAL, "score_round: call ut_gp_fit first");
  UT_CHECK(c, c->gp_d == c->space.n_feat, UT_EINVAL, "score_round: GP feature width != space feature width");
  UT_CHECK(c, m >= 1 && ga && acq && cand_base >= 0 && k >= 1, UT_EINVAL, "score_round_ga: bad arguments");
  UT_CHECK(c, ga->max_retries >= 1 && ga->max_retries <= 15, UT_EINVAL, "propose_ga: max_retries must be in [1, 15]");
  UT_CHECK(c, ga->must_mutate_count >= 0 && ga->must_mutate_count <= c->space.P, UT_EINVAL,
           "propose_ga: must_mutate_count out of range");
  UT_CHECK(c, ga->op >= 0 && ga->op < 256, UT_EINVAL, "propose_ga: op must fit 8 bits");
  UT_CHECK(c, ga->crossover >= UT_X_NONE && ga->crossover <= UT_X_PMX, UT_EINVAL, "propose_ga: bad crossover");
  const int64_t ld = ((m + 127) / 128) * 128;
  int rc;
  if ((rc = ensure(c, c->r_values, (size_t)c->space.ncols * ld))) return rc;
  if ((rc = ensure(c, c->r_digest, (size_t)8 * ld))) return rc;
  if ((rc = ensure(c, c->r_dup, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_inval, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_mu, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_var, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_score, (size_t)ld))) return rc;
  if ((rc = ensure(c, c->r_topk_idx, (size_t)k))) return rc;
  if ((rc = ensure(c, c->r_topk_score, (size_t)k))) return rc;
  c->r_ld = ld;
  c->r_m = m;
  c->r_feat_valid = false;
  timing_begin(c);
  if ((rc = gp_fit_prefit(c))) return rc;   // (as score_round_de_impl)
  if ((rc = launch_ga(c, ga, parent1, parent2, round_, cand_base, m, c->r_values.p, ld, c->r_inval.p))) return rc;
  if ((rc = gp_fit_flush(c))) return rc;
  mark(c, "propose");
  // fork right after the proposal: forked after K* instead (beside the int8
  // variance GEMM) the hash ran 106 ms where it runs 79 beside encode + K*, C4
  // 147.5 -> 156.5 ms (scripts/ab/r05_ga_fork.sh)
  UT_HIP(c, hipEventRecord(c->ev_fork, c->stream));
  UT_HIP(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
  {
    StreamScope on_side(c, c->side);
    mark(c, "");
    rc = parent1 ? launch_hash_parent(c, c->r_values.p, ld, m, parent1, c->r_digest.p)
                 : launch_hash(c, c->r_values.p, ld, m, c->r_digest.p);
    if (rc) return rc;
    mark(c, "hash");
    if ((rc = launch_dedup(c, c->r_digest.p, m, c->r_dup.p))) return rc;
    if ((rc = launch_mask_or(c, c->r_dup.p, c->r_inval.p, m))) return rc;
    mark(c, "dedup");
    UT_HIP(c, hipEventRecord(c->ev_join, c->side));
  }
  if ((rc = gp_encode_scaled(c, c->r_values.p, ld, m))) return rc;
  mark(c, "encode");
  if ((rc = gp_score_impl(c, nullptr, ld, m, acq, c->r_dup.p, c->r_mu.p, c->r_var.p, c->r_score.p, c->ev_join)))
    return rc;
  if ((rc = topk_impl(c, c->r_score.p, c->r_dup.p, m, cand_base, k, c->r_topk_idx.p, c->r_topk_score.p))) return rc;
  mark(c, "topk");
  if ((rc = round_outputs(c, out, ld, cand_base, k))) return rc;
  mark(c, "outputs");
  return timing_end(c);
}

int ut_round_buffers(ut_ctx* c, double** values, double** features, uint32_t** digests, uint8_t** dup,
                     double** mu, double** var, double** score, int64_t* ld) {
  if (!c) return UT_EINVAL;
  if (values) *values = c->r_values.p;
  if (features) *features = c->r_feat_valid ? c->r_feat.p : nullptr;   // dense rounds keep no feature matrix
  if (digests) *digests = c->r_digest.p;
  if (dup) *dup = c->r_dup.p;
  if (mu) *mu = c->r_mu.p;
  if (var) *var = c->r_var.p;
  if (score) *score = c->r_score.p;
  if (ld) *ld = c->r_ld;
  return 0;
}

int ut_set_timing(ut_ctx* c, int32_t on) {
  if (!c) return UT_EINVAL;
  int rc = timing_collect(c, false);  // a (re)start discards what was recorded
  c->timing.totals.clear();
  c->timing.round = 0;
  c->timing.on = on != 0;
  return rc;
}

int ut_stage_time(ut_ctx* c, const char* stage, double* ms) {
  if (!c || !stage || !ms) return UT_EINVAL;
  int rc = timing_collect(c, true);
  if (rc) return rc;
  for (auto& e : c->timing.totals)
    if (e.first == stage && e.second.second > 0) {
      *ms = e.second.first / (double)e.second.second;
      return 0;
    }
  return set_err(c, UT_EINVAL, std::string("no timing for stage ") + stage);
}

}  // extern "C"
