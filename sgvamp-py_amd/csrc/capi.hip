// C ABI of libsgvamp_hip.so (declared in include/sgvamp_hip.h), part 1 of the
// host side: error handling, the A/B switch gate, context lifetime, host <->
// device staging (pinned copies, probe uploads), solver settings, vectors, the
// device data generator's entry points, output copies, timers.  The other
// parts: exchange.hip, ldplan.hip, solver.hip (ctx.h lists them).
#include "ctx.h"

static thread_local std::string g_last_err;

// A/B tuning switches: an environment override is honoured only with
// SGV_AB=1 (and then announced once on stderr); without it a set override is
// ignored with a warning, so no stray variable changes a production run.
const char* sgv::ab_env(const char* name) {
  const char* v = std::getenv(name);
  if (!v) return nullptr;
  const char* ab = std::getenv("SGV_AB");
  const bool on = ab && ab[0] == '1';
  static std::mutex mu;
  static std::vector<std::string> told;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (std::find(told.begin(), told.end(), name) == told.end()) {
      told.emplace_back(name);
      std::fprintf(stderr, on ? "[sgvamp] A/B override %s=%s active (SGV_AB=1)\n"
                              : "[sgvamp] %s=%s ignored: A/B overrides need SGV_AB=1\n",
                   name, v);
    }
  }
  return on ? v : nullptr;
}

// ---------------------------------------------------------------------------
// error handling
// ---------------------------------------------------------------------------
int fail(sgv_ctx* c, int code, const char* fmt, ...){
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  g_last_err = buf;
  return code;
}

// Host wait for the ctx stream: record an event and spin on it.  The default
// hipStreamSynchronize may park the thread and wake it late (measured on
// MI355X: ~10 ms extra per wait), and the CG loop waits once per iteration.
int stream_wait(sgv_ctx* c){
  HIPCHK(hipEventRecord(c->ev_sync, c->st));
  hipError_t e;
  while ((e = hipEventQuery(c->ev_sync)) == hipErrorNotReady) {
    __builtin_ia32_pause();
  }
  if (e != hipSuccess)
    return fail(c, SGV_ERR_HIP, "stream wait: %s", hipGetErrorString(e));
  return SGV_OK;
}

void resolve_timers(sgv_ctx* c){
  for (size_t i = 0; i < c->pending.size(); ++i) {
    const auto& pr = c->pending[i];
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
      c->ld_ms += ms;
      if (c->pending_wide[i]) c->ld_ms_wide += ms;
    }
    c->evpool.push_back(pr.first);
    c->evpool.push_back(pr.second);
  }
  c->pending.clear();
  c->pending_wide.clear();
  for (auto& pr : c->xpending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) c->xchg_ms += ms;
    c->evpool.push_back(pr.first);
    c->evpool.push_back(pr.second);
  }
  c->xpending.clear();
  for (auto& pr : c->gpending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) c->host_wait_ms += ms;
    c->evpool.push_back(pr.first);
    c->evpool.push_back(pr.second);
  }
  c->gpending.clear();
  for (auto& pr : c->empending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
      c->em_ms += ms;
      c->em_loops_timed += 1.0;
    }
    c->evpool.push_back(pr.first);
    c->evpool.push_back(pr.second);
  }
  c->empending.clear();
}

int event_pair(sgv_ctx* c, hipEvent_t* e0, hipEvent_t* e1){
  if (c->evpool.size() < 2) {
    HIPCHK(hipEventCreate(e0));
    HIPCHK(hipEventCreate(e1));
  } else {
    *e0 = c->evpool.back();
    c->evpool.pop_back();
    *e1 = c->evpool.back();
    c->evpool.pop_back();
  }
  return SGV_OK;
}

int ensure_stage(sgv_ctx* c, size_t bytes){
  if (bytes <= c->stage_bytes) return SGV_OK;
  if (c->d_stage) HIPCHK(hipFree(c->d_stage));
  c->d_stage = nullptr;
  HIPCHK(hipMalloc(&c->d_stage, bytes));
  c->stage_bytes = bytes;
  return SGV_OK;
}

int ensure_hstage(sgv_ctx* c, size_t bytes){
  if (bytes <= c->h_stage_bytes) return SGV_OK;
  if (c->h_stage) HIPCHK(hipHostFree(c->h_stage));
  c->h_stage = nullptr;
  HIPCHK(hipHostMalloc(&c->h_stage, bytes));
  c->h_stage_bytes = bytes;
  return SGV_OK;
}

// host (pageable) -> pinned -> device staging buffer; returns when the copy
// has landed (the pinned buffer may be reused right away)
static int h2d(sgv_ctx* c, const void* host, size_t bytes) {
  CHK(ensure_stage(c, std::max<size_t>(bytes, 8)));
  CHK(ensure_hstage(c, std::max<size_t>(bytes, 8)));
  std::memcpy(c->h_stage, host, bytes);
  HIPCHK(hipMemcpyAsync(c->d_stage, c->h_stage, bytes, hipMemcpyHostToDevice, c->st));
  return stream_wait(c);
}

// host half of a probe upload: the next pinned slot, once its previous copy
// has finished (long done), takes the K x Mloc probes; returns the slot or -1.
// Needs the buffers (probe_cap) in place; touches nothing a running step uses.
int probe_stage(sgv_ctx* c, const int8_t* probes){
  const int slot = c->probe_slot.fetch_xor(1);
  if (hipEventSynchronize(c->ev_probe[slot]) != hipSuccess) {
    fail(c, SGV_ERR_HIP, "probe slot wait failed");
    return -1;
  }
  std::memcpy(c->h_probe[slot], probes, (size_t)c->K * c->Mloc);
  return slot;
}
// K x Mloc int8 probes -> d_probe slot, copied on the copy stream (no host wait);
// returns the slot.  A slot's device half is consumed by the unpack kernels of
// its step (ev_unpk) and reused two uploads later.
int probe_upload(sgv_ctx* c, const int8_t* probes, int* slot_out){
  const size_t bytes = std::max<size_t>((size_t)c->K * c->Mloc, 8);
  if (bytes > c->probe_cap) {
    CHK(stream_wait(c));
    HIPCHK(hipStreamSynchronize(c->st_copy));
    for (int i = 0; i < 2; ++i) {
      if (c->h_probe[i]) HIPCHK(hipHostFree(c->h_probe[i]));
      c->h_probe[i] = nullptr;
      HIPCHK(hipHostMalloc(&c->h_probe[i], bytes));
      if (!c->ev_probe[i]) HIPCHK(hipEventCreateWithFlags(&c->ev_probe[i], hipEventDisableTiming));
      if (!c->ev_unpk[i]) HIPCHK(hipEventCreateWithFlags(&c->ev_unpk[i], hipEventDisableTiming));
    }
    if (c->d_probe) HIPCHK(hipFree(c->d_probe));
    c->d_probe = nullptr;
    HIPCHK(hipMalloc(&c->d_probe, 2 * bytes));
    c->probe_cap.store(bytes, std::memory_order_release);
  }
  const int slot = probe_stage(c, probes);
  if (slot < 0) return SGV_ERR_HIP;
  return probe_issue(c, slot, slot_out);
}

// device half of an upload staged by probe_stage: behind the slot's previous
// unpack (ev_unpk), on the copy stream
int probe_issue(sgv_ctx* c, int slot, int* slot_out){
  HIPCHK(hipStreamWaitEvent(c->st_copy, c->ev_unpk[slot], 0));
  HIPCHK(hipMemcpyAsync(c->d_probe + slot * c->probe_cap, c->h_probe[slot],
                        (size_t)c->K * c->Mloc, hipMemcpyHostToDevice, c->st_copy));
  HIPCHK(hipEventRecord(c->ev_probe[slot], c->st_copy));
  *slot_out = slot;
  return SGV_OK;
}

int upload_vec(sgv_ctx* c, const double* host, double* dpad){
  CHK(h2d(c, host, sizeof(double) * c->Mloc));
  HIPCHK(launch_unpack(c->d_ch, c->nch, c->d_ch_doff, (const double*)c->d_stage, dpad, c->st));
  return SGV_OK;
}

int download_vec(sgv_ctx* c, const double* dpad, double* host){
  const size_t bytes = sizeof(double) * std::max<int64_t>(c->Mloc, 1);
  CHK(ensure_stage(c, bytes));
  CHK(ensure_hstage(c, bytes));
  HIPCHK(launch_pack(c->d_ch, c->nch, c->d_ch_doff, dpad, (double*)c->d_stage, c->st));
  HIPCHK(hipMemcpyAsync(c->h_stage, c->d_stage, sizeof(double) * c->Mloc, hipMemcpyDeviceToHost,
                        c->st));
  CHK(stream_wait(c));
  std::memcpy(host, c->h_stage, sizeof(double) * c->Mloc);
  return SGV_OK;
}

bool host_any(const double* v, int64_t n){
  for (int64_t i = 0; i < n; ++i)
    if (v[i] != 0.0) return true;
  return false;
}

// ---------------------------------------------------------------------------
// lifetime
// ---------------------------------------------------------------------------
extern "C" int sgv_create(int device, int K, int nld, const int* ld_of, int nblk,
                          const int64_t* blk_sizes, int blk0, int nblk_global, int64_t M_total,
                          sgv_ctx** out) {
  sgv_ctx* c = nullptr;
  if (!out) return fail(nullptr, SGV_ERR_ARG, "out is null");
  *out = nullptr;
  if (K < 1 || K > MAXCOH) return fail(nullptr, SGV_ERR_ARG, "K=%d outside [1,%d]", K, MAXCOH);
  if (nld < 1 || nld > K) return fail(nullptr, SGV_ERR_ARG, "nld=%d outside [1,K]", nld);
  if (nblk < 1 || !blk_sizes) return fail(nullptr, SGV_ERR_ARG, "need >= 1 LD block");
  for (int k = 0; k < K; ++k)
    if (!ld_of || ld_of[k] < 0 || ld_of[k] >= nld)
      return fail(nullptr, SGV_ERR_ARG, "ld_of[%d] invalid", k);
  for (int b = 0; b < nblk; ++b)
    if (blk_sizes[b] < 1 || blk_sizes[b] > (int64_t)1 << 30)
      return fail(nullptr, SGV_ERR_ARG, "block %d size %lld invalid", b,
                  (long long)blk_sizes[b]);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(nullptr, SGV_ERR_HIP, "no HIP device visible");
  if (device < 0 || device >= ndev)
    return fail(nullptr, SGV_ERR_ARG, "device %d outside [0,%d)", device, ndev);

  c = new sgv_ctx();
  c->mfma_min = mfma_min_default();
  c->dev = device;
  c->K = K;
  c->nld = nld;
  c->ld_of.assign(ld_of, ld_of + K);
  c->nblk = nblk;
  c->blk0 = blk0;
  c->nblk_global = nblk_global;
  c->Mtot = M_total;
  c->Ncoh.assign(K, 1.0);
  int rc = SGV_OK;
  auto cleanup = [&](int code) {
    sgv_destroy(c);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return cleanup(fail(nullptr, SGV_ERR_HIP, "hipSetDevice"));
  (void)hipSetDeviceFlags(hipDeviceScheduleSpin);   // best effort; waits spin anyway
  if (hipEventCreateWithFlags(&c->ev_sync, hipEventDisableTiming) != hipSuccess)
    return cleanup(fail(nullptr, SGV_ERR_HIP, "hipEventCreate"));
  if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(nullptr, SGV_ERR_HIP, "hipStreamCreate"));
  if (hipStreamCreateWithFlags(&c->st_copy, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(nullptr, SGV_ERR_HIP, "hipStreamCreate"));
  if (hipStreamCreateWithFlags(&c->st_fin, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(nullptr, SGV_ERR_HIP, "hipStreamCreate"));
  for (int g = 0; g < MAXGRP; ++g)
    if (hipEventCreateWithFlags(&c->ev_grp[g], hipEventDisableTiming) != hipSuccess)
      return cleanup(fail(nullptr, SGV_ERR_HIP, "hipEventCreate"));
  if (hipEventCreateWithFlags(&c->ev_fin, hipEventDisableTiming) != hipSuccess)
    return cleanup(fail(nullptr, SGV_ERR_HIP, "hipEventCreate"));

  // marker layout
  int64_t off = 0, voff = 0;
  for (int b = 0; b < nblk; ++b) {
    c->bn.push_back(blk_sizes[b]);
    c->boff.push_back(off);
    c->bvoff.push_back(voff);
    c->lda.push_back(round_up(blk_sizes[b], PADV));
    off += blk_sizes[b];
    voff += round_up(blk_sizes[b], PADV);
  }
  c->Mloc = off;
  c->Mpad = std::max<int64_t>(voff, PADV);

  // chunks and row groups (restart at every block start)
  std::vector<ChunkDesc> ch;
  std::vector<int64_t> chdoff;
  std::vector<int> chb(nblk + 1, 0);
  for (int b = 0; b < nblk; ++b) {
    chb[b] = (int)ch.size();
    for (int64_t o = 0; o < c->bn[b]; o += CHUNK) {
      ch.push_back(ChunkDesc{c->bvoff[b] + o, (int32_t)std::min<int64_t>(CHUNK, c->bn[b] - o), b});
      chdoff.push_back(c->boff[b] + o);
    }
  }
  chb[nblk] = (int)ch.size();
  c->nch = (int)ch.size();

#define CREATE_HIP(expr)                                                          \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return cleanup(fail(nullptr, SGV_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_))); \
  } while (0)

  CREATE_HIP(hipMalloc(&c->d_ch, sizeof(ChunkDesc) * ch.size()));
  CREATE_HIP(hipMemcpy(c->d_ch, ch.data(), sizeof(ChunkDesc) * ch.size(), hipMemcpyHostToDevice));
  CREATE_HIP(hipMalloc(&c->d_ch_doff, sizeof(int64_t) * chdoff.size()));
  CREATE_HIP(hipMemcpy(c->d_ch_doff, chdoff.data(), sizeof(int64_t) * chdoff.size(),
                       hipMemcpyHostToDevice));
  CREATE_HIP(hipMalloc(&c->d_ch_begin, sizeof(int) * chb.size()));
  CREATE_HIP(hipMemcpy(c->d_ch_begin, chb.data(), sizeof(int) * chb.size(), hipMemcpyHostToDevice));

  // LD descriptors
  c->ldb.assign(nld, std::vector<LdBlock>(nblk));
  c->plan.assign(nld, LdPlan());
  c->cpl.assign(nld, std::vector<LdCoupling>());
  c->rank_blk0 = {blk0, blk0 + nblk};   // one rank until a communicator says otherwise
  for (int l = 0; l < nld; ++l) {
    BlkDesc* d = nullptr;
    CREATE_HIP(hipMalloc(&d, sizeof(BlkDesc) * nblk));
    std::vector<BlkDesc> h(nblk);
    for (int b = 0; b < nblk; ++b) h[b] = BlkDesc{nullptr, c->lda[b], c->bn[b], c->bvoff[b]};
    CREATE_HIP(hipMemcpy(d, h.data(), sizeof(BlkDesc) * nblk, hipMemcpyHostToDevice));
    c->d_blks.push_back(d);
  }

  // vectors: r, r1, r2, U (K each); xhat1, x0; X, X0, Rr, P, Q, RX0, Y, RXp (2K each);
  // S: 5 * MAXC scratch columns for the operator-seam entry points
  const int nvec = 4 * K + 2 + 16 * K + 5 * MAXC;
  const size_t vbytes = sizeof(double) * (size_t)c->Mpad * nvec;
  CREATE_HIP(hipMalloc(&c->pool, vbytes));
  CREATE_HIP(hipMemset(c->pool, 0, vbytes));
  double* p = c->pool;
  auto take = [&](std::vector<double*>& v, int n) {
    for (int i = 0; i < n; ++i) {
      v.push_back(p);
      p += c->Mpad;
    }
  };
  take(c->r, K);
  take(c->r1, K);
  take(c->r2, K);
  take(c->U, K);
  c->xhat1 = p;
  p += c->Mpad;
  c->x0 = p;
  p += c->Mpad;
  take(c->X, 2 * K);
  take(c->X0, 2 * K);
  take(c->Rr, 2 * K);
  take(c->P, 2 * K);
  take(c->Q, 2 * K);
  take(c->RX0, 2 * K);
  take(c->Y, 2 * K);
  take(c->RXp, 2 * K);
  take(c->S, 5 * MAXC);

  const size_t part_n = (size_t)c->nch * MAXNV;
  CREATE_HIP(hipMalloc(&c->d_part, sizeof(double) * part_n));
  c->part_cap = part_n;
  c->nbmax = nblk;
  CREATE_HIP(hipMalloc(&c->d_bsum, sizeof(double) * (size_t)nblk * MAXNV));
  CREATE_HIP(hipMalloc(&c->d_counts, sizeof(int)));
  CREATE_HIP(hipMemcpy(c->d_counts, &nblk, sizeof(int), hipMemcpyHostToDevice));
  CREATE_HIP(hipMalloc(&c->d_tot, sizeof(double) * 64));
  CREATE_HIP(hipMalloc(&c->d_pq, sizeof(double) * 2 * MAXC));
  // >= (MAXL + 1) * (MAXL + 1): the MLE Jacobian's batched sums (mle_jacobian)
  CREATE_HIP(hipHostMalloc(&c->h_tot, sizeof(double) * std::max(128, K), hipHostMallocCoherent));
  CREATE_HIP(hipMalloc(&c->d_cgs, sizeof(CgState)));
  CREATE_HIP(hipMalloc(&c->d_rhonew, sizeof(double) * MAXC));
  CREATE_HIP(hipHostMalloc(&c->h_cgm, sizeof(CgState) * CG_RING, hipHostMallocCoherent));
  CREATE_HIP(hipHostMalloc(&c->h_cgi, sizeof(CgState)));
  for (int i = 0; i < CG_RING; ++i)
    CREATE_HIP(hipEventCreateWithFlags(&c->ev_cg[i], hipEventDisableTiming));
  CREATE_HIP(hipEventCreateWithFlags(&c->ev_den, hipEventDisableTiming));
  CREATE_HIP(hipMalloc(&c->d_ems, sizeof(EmState)));
  CREATE_HIP(hipMalloc(&c->d_emtot, sizeof(double) * MAXNV));
  CREATE_HIP(hipMalloc(&c->d_emtab, sizeof(double) * std::max(K, MAXK) * EM_TAB));
  c->chain.gam1.assign(K, 0.0);
  c->chain.gamw.assign(K, 0.0);
  c->chain.alpha1.assign(K, 0.0);
  c->chain.alpha2.assign(K, 0.0);
  CREATE_HIP(hipHostMalloc(&c->h_emm, sizeof(EmState) * CG_RING, hipHostMallocCoherent));
  CREATE_HIP(hipHostMalloc(&c->h_emi, sizeof(EmState)));
  for (int i = 0; i < CG_RING; ++i)
    CREATE_HIP(hipEventCreateWithFlags(&c->ev_em[i], hipEventDisableTiming));
  c->cg_pipe = cg_pipe_default();
  c->cg_exact = cg_exact_default();
  c->xnz.assign(2 * K, 0);
  c->rx0_valid.assign(2 * K, 0);
#undef CREATE_HIP
  (void)rc;
  *out = c;
  return SGV_OK;
}

extern "C" void sgv_destroy(sgv_ctx* c) {
  if (!c) return;
  if (c->worker.joinable()) {
    for (auto& j : c->jobs)
      while (j.state.load() == 1 || j.state.load() == 2) __builtin_ia32_pause();
    {
      std::lock_guard<std::mutex> lk(c->wmu);
      c->worker_quit = true;
    }
    c->wcv.notify_all();
    c->worker.join();
  }
  (void)hipSetDevice(c->dev);
  if (c->st) (void)hipStreamSynchronize(c->st);
  if (c->st_fin) (void)hipStreamSynchronize(c->st_fin);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->h_bsum) (void)hipHostFree(c->h_bsum);
  if (c->h_bsum_all) (void)hipHostFree(c->h_bsum_all);
  for (auto& v : c->ldb)
    for (LdBlock& lb : v) free_block(lb);
  for (LdPlan& pl : c->plan) free_plan(pl);
  for (auto& v : c->cpl)
    for (LdCoupling& q : v) {
      if (q.d_up) (void)hipFree(q.d_up);
      if (q.d_lo) (void)hipFree(q.d_lo);
    }
  if (c->d_cpbuf) (void)hipFree(c->d_cpbuf);
  if (c->d_halo) (void)hipFree(c->d_halo);
  if (c->h_halo) (void)hipHostFree(c->h_halo);
  if (c->d_rowpart) (void)hipFree(c->d_rowpart);
  if (c->d_whead) (void)hipFree(c->d_whead);
  if (c->d_wcarry) (void)hipFree(c->d_wcarry);
  if (c->d_colpart) (void)hipFree(c->d_colpart);
  if (c->d_pk) (void)hipFree(c->d_pk);
  if (c->d_out) (void)hipFree(c->d_out);
  for (int i = 0; i < 2; ++i) {

    if (c->h_probe[i]) (void)hipHostFree(c->h_probe[i]);
    if (c->ev_probe[i]) (void)hipEventDestroy(c->ev_probe[i]);
  }
  if (c->d_probe) (void)hipFree(c->d_probe);
  if (c->h_met) (void)hipHostFree(c->h_met);
  if (c->ev_met) (void)hipEventDestroy(c->ev_met);
  for (BlkDesc* d : c->d_blks) (void)hipFree(d);
  (void)hipFree(c->d_ch);
  (void)hipFree(c->d_ch_doff);
  (void)hipFree(c->d_ch_begin);
  (void)hipFree(c->pool);
  (void)hipFree(c->d_part);
  if (c->d_part2) (void)hipFree(c->d_part2);
  (void)hipFree(c->d_bsum);
  if (c->d_bsum_all) (void)hipFree(c->d_bsum_all);
  (void)hipFree(c->d_counts);
  (void)hipFree(c->d_tot);
  (void)hipFree(c->d_pq);
  if (c->h_tot) (void)hipHostFree(c->h_tot);
  if (c->d_cgs) (void)hipFree(c->d_cgs);
  if (c->d_rhonew) (void)hipFree(c->d_rhonew);
  if (c->h_cgm) (void)hipHostFree(c->h_cgm);
  if (c->h_cgi) (void)hipHostFree(c->h_cgi);
  for (hipEvent_t e : c->ev_cg)
    if (e) (void)hipEventDestroy(e);
  if (c->d_ems) (void)hipFree(c->d_ems);
  if (c->d_chg) (void)hipFree(c->d_chg);
  if (c->d_chg_begin) (void)hipFree(c->d_chg_begin);
  if (c->d_partg) (void)hipFree(c->d_partg);
  if (c->d_r1send) (void)hipFree(c->d_r1send);
  if (c->d_r1g) (void)hipFree(c->d_r1g);
  if (c->h_r1send) (void)hipHostFree(c->h_r1send);
  if (c->h_r1g) (void)hipHostFree(c->h_r1g);
  if (c->d_emtot) (void)hipFree(c->d_emtot);
  if (c->d_emtab) (void)hipFree(c->d_emtab);
  if (c->d_inner) (void)hipFree(c->d_inner);
  if (c->h_emm) (void)hipHostFree(c->h_emm);
  if (c->h_emi) (void)hipHostFree(c->h_emi);
  for (hipEvent_t e : c->ev_em)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_den) (void)hipEventDestroy(c->ev_den);
  if (c->d_stage) (void)hipFree(c->d_stage);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  for (auto* v : {&c->pending, &c->xpending, &c->gpending})
    for (auto& pr : *v) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (hipEvent_t e : c->evpool) (void)hipEventDestroy(e);
  if (c->ev_sync) (void)hipEventDestroy(c->ev_sync);
  if (c->st_copy) (void)hipStreamSynchronize(c->st_copy);
  for (int i = 0; i < 2; ++i) {
    if (c->ev_unpk[i]) (void)hipEventDestroy(c->ev_unpk[i]);

  }
  for (int i = 0; i < NOUT_SLOTS; ++i) {
    if (c->h_out[i]) (void)hipHostFree(c->h_out[i]);
    if (c->ev_out[i]) (void)hipEventDestroy(c->ev_out[i]);
    if (c->ev_pack[i]) (void)hipEventDestroy(c->ev_pack[i]);
  }
  if (c->st_fin) (void)hipStreamSynchronize(c->st_fin);
  for (hipEvent_t e : c->ev_grp)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_fin) (void)hipEventDestroy(c->ev_fin);
  if (c->st_fin) (void)hipStreamDestroy(c->st_fin);
  if (c->st_copy) (void)hipStreamDestroy(c->st_copy);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
}

extern "C" const char* sgv_last_error(const sgv_ctx* c) {
  return c ? c->err.c_str() : g_last_err.c_str();
}

// Start a new infer() on the same context (src/sgvamp.py:198-217 resets r1,
// xhat1, xhat2, Sigma2_u_prev and the scalars every call): every solver vector
// except r, r1 and x0 is zeroed, the warm-start flags and the chained-step
// inputs are cleared.  LD blocks, ridge and cohort sizes stay.
extern "C" int sgv_reset_solver(sgv_ctx* c) {
  ENTER(c);
  if (c->job_ended != c->job_begun)
    return fail(c, SGV_ERR_STATE, "sgv_reset_solver: a step is still queued");
  const size_t n = sizeof(double) * (size_t)c->Mpad;
  for (auto* v : {&c->r2, &c->U, &c->X, &c->X0, &c->Rr, &c->P, &c->Q, &c->RX0, &c->Y, &c->RXp})
    for (double* d : *v) HIPCHK(hipMemsetAsync(d, 0, n, c->st));
  HIPCHK(hipMemsetAsync(c->xhat1, 0, n, c->st));
  CHK(stream_wait(c));
  std::fill(c->xnz.begin(), c->xnz.end(), 0);
  std::fill(c->rx0_valid.begin(), c->rx0_valid.end(), 0);
  c->chain.valid = 0;
  c->met_pending = 0;
  return SGV_OK;
}

extern "C" int sgv_set_mle_gam(sgv_ctx* c, double gam) {
  ENTER(c);
  c->mle_gam = gam;
  return SGV_OK;
}

extern "C" int sgv_set_rs_recurrence(sgv_ctx* c, int on) {
  ENTER(c);
  c->rs_rec = on ? 1 : 0;
  std::fill(c->rx0_valid.begin(), c->rx0_valid.end(), 0);   // re-derive R_s x0 once
  return SGV_OK;
}

extern "C" int sgv_set_cg_pipeline(sgv_ctx* c, int on) {
  ENTER(c);
  c->cg_pipe = on ? 1 : 0;
  return SGV_OK;
}

extern "C" int sgv_set_cg_exact(sgv_ctx* c, int mode) {
  ENTER(c);
  if (mode < -1 || mode > 1) return fail(c, SGV_ERR_ARG, "cg exact mode must be -1, 0 or 1");
  const int forced = cg_exact_default();   // an A/B override wins
  c->cg_exact = forced >= 0 ? forced : mode;
  return SGV_OK;
}

extern "C" int sgv_set_mfma_min(sgv_ctx* c, int nc_min) {
  ENTER(c);
  if (nc_min < 0) return fail(c, SGV_ERR_ARG, "nc_min must be >= 0");
  c->mfma_min = nc_min;
  return SGV_OK;
}

extern "C" int sgv_set_cohort_n(sgv_ctx* c, int k, double N) {
  ENTER(c);
  if (k < 0 || k >= c->K) return fail(c, SGV_ERR_ARG, "cohort %d", k);
  c->Ncoh[k] = N;
  return SGV_OK;
}

static double* vec_ptr(sgv_ctx* c, int which, int k) {
  const bool kok = k >= 0 && k < c->K;
  switch (which) {
    case SGV_VEC_R: return kok ? c->r[k] : nullptr;
    case SGV_VEC_R1: return kok ? c->r1[k] : nullptr;
    case SGV_VEC_XHAT1: return c->xhat1;
    case SGV_VEC_XHAT2: return kok ? c->X[2 * k] : nullptr;
    case SGV_VEC_SIG2U: return kok ? c->X[2 * k + 1] : nullptr;
    case SGV_VEC_X0: return c->x0;
    default: return nullptr;
  }
}

extern "C" int sgv_set_vector(sgv_ctx* c, int which, int k, const double* host) {
  ENTER(c);
  double* d = vec_ptr(c, which, k);
  if (!d || !host) return fail(c, SGV_ERR_ARG, "sgv_set_vector: which=%d k=%d", which, k);
  CHK(upload_vec(c, host, d));
  CHK(stream_wait(c));
  if (which == SGV_VEC_XHAT2 || which == SGV_VEC_SIG2U) {
    const int col = 2 * k + (which == SGV_VEC_SIG2U);
    c->xnz[col] = host_any(host, c->Mloc);
    c->rx0_valid[col] = 0;
  }
  return SGV_OK;
}

extern "C" int sgv_get_vector(sgv_ctx* c, int which, int k, double* host) {
  ENTER(c);
  double* d = vec_ptr(c, which, k);
  if (!d || !host) return fail(c, SGV_ERR_ARG, "sgv_get_vector: which=%d k=%d", which, k);
  return download_vec(c, d, host);
}

// ---------------------------------------------------------------------------
// synthetic inputs
// ---------------------------------------------------------------------------
struct SynthBufs {
  double *G = nullptr, *mean = nullptr, *sd = nullptr, *vec = nullptr, *g = nullptr;
  ~SynthBufs() {
    if (G) (void)hipFree(G);
    if (mean) (void)hipFree(mean);
    if (sd) (void)hipFree(sd);
    if (vec) (void)hipFree(vec);
    if (g) (void)hipFree(g);
  }
};

extern "C" int sgv_synth_ld_g(sgv_ctx* c, int ld, uint64_t seed, int64_t marker0, int Nsamp,
                              const double* beta, double* g_out) {
  ENTER(c);
  if (ld >= c->nld || Nsamp < 2 || !beta || !g_out)
    return fail(c, SGV_ERR_ARG, "sgv_synth_ld_g: bad arguments");
  const int64_t nmax = *std::max_element(c->bn.begin(), c->bn.end());
  const int ldg = (int)round_up(Nsamp, 16);
  SynthBufs sb;
  HIPCHK(hipMalloc(&sb.G, sizeof(double) * (size_t)nmax * ldg));
  HIPCHK(hipMalloc(&sb.mean, sizeof(double) * nmax));
  HIPCHK(hipMalloc(&sb.sd, sizeof(double) * nmax));
  HIPCHK(hipMalloc(&sb.vec, sizeof(double) * std::max<int64_t>(c->Mloc, 1)));
  HIPCHK(hipMalloc(&sb.g, sizeof(double) * Nsamp));
  CHK(h2d(c, beta, sizeof(double) * c->Mloc));
  HIPCHK(hipMemcpyAsync(sb.vec, c->d_stage, sizeof(double) * c->Mloc, hipMemcpyDeviceToDevice,
                        c->st));
  for (int b = 0; b < c->nblk; ++b) {
    const int n = (int)c->bn[b];
    const int64_t gm0 = marker0 + c->boff[b];
    HIPCHK(launch_geno_stats(seed, gm0, n, Nsamp, sb.mean, sb.sd, c->st));
    if (ld >= 0) {
      CHK(ld_alloc(c, ld, b, c->packing));    // R = G G^T is exactly symmetric
      const LdBlock& lb = c->ldb[ld][b];
      HIPCHK(launch_geno_G(seed, gm0, n, Nsamp, ldg, sb.mean, sb.sd, sb.G, c->st));
      HIPCHK(launch_syrk_nt(sb.G, n, Nsamp, ldg, lb.ptr, c->lda[b], lb.fmt, lb.d_poff, lb.d_pw,
                            c->st));
    }
    HIPCHK(launch_g_accum(seed, gm0, n, Nsamp, sb.mean, sb.sd, sb.vec + c->boff[b], sb.g, c->st));
    CHK(ensure_hstage(c, sizeof(double) * Nsamp));
    HIPCHK(hipMemcpyAsync(c->h_stage, sb.g, sizeof(double) * Nsamp, hipMemcpyDeviceToHost, c->st));
    CHK(stream_wait(c));
    std::memcpy(g_out + (size_t)b * Nsamp, c->h_stage, sizeof(double) * Nsamp);
  }
  std::fill(c->rx0_valid.begin(), c->rx0_valid.end(), 0);
  return SGV_OK;
}

extern "C" int sgv_synth_r(sgv_ctx* c, int k, uint64_t seed, int64_t marker0, int Nsamp,
                           const double* y) {
  ENTER(c);
  if (k < 0 || k >= c->K || Nsamp < 2 || !y) return fail(c, SGV_ERR_ARG, "sgv_synth_r: bad arguments");
  const int64_t nmax = *std::max_element(c->bn.begin(), c->bn.end());
  const int ldg = (int)round_up(Nsamp, 16);
  SynthBufs sb;
  HIPCHK(hipMalloc(&sb.G, sizeof(double) * (size_t)nmax * ldg));
  HIPCHK(hipMalloc(&sb.mean, sizeof(double) * nmax));
  HIPCHK(hipMalloc(&sb.sd, sizeof(double) * nmax));
  HIPCHK(hipMalloc(&sb.g, sizeof(double) * Nsamp));
  CHK(h2d(c, y, sizeof(double) * Nsamp));
  HIPCHK(hipMemcpyAsync(sb.g, c->d_stage, sizeof(double) * Nsamp, hipMemcpyDeviceToDevice, c->st));
  for (int b = 0; b < c->nblk; ++b) {
    const int n = (int)c->bn[b];
    const int64_t gm0 = marker0 + c->boff[b];
    HIPCHK(launch_geno_stats(seed, gm0, n, Nsamp, sb.mean, sb.sd, c->st));
    HIPCHK(launch_geno_G(seed, gm0, n, Nsamp, ldg, sb.mean, sb.sd, sb.G, c->st));
    HIPCHK(launch_row_dot(sb.G, n, Nsamp, ldg, sb.g, c->r[k] + c->bvoff[b], c->st));
  }
  CHK(stream_wait(c));
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// per-iteration outputs without a host wait (src/sgvamp.py:281,283)
// ---------------------------------------------------------------------------
extern "C" int sgv_outputs_begin(sgv_ctx* c, int slot) {
  ENTER(c);
  if (slot < 0 || slot >= NOUT_SLOTS) return fail(c, SGV_ERR_ARG, "slot must be 0, 1 or 2");
  const size_t n = (size_t)std::max<int64_t>(c->Mloc, 1);
  const size_t bytes = sizeof(double) * n * (c->K + 1);
  if (!c->d_out) {   // a device staging half and a pinned buffer per slot
    HIPCHK(hipMalloc(&c->d_out, NOUT_SLOTS * bytes));
    for (int i = 0; i < NOUT_SLOTS; ++i) {
      HIPCHK(hipHostMalloc(&c->h_out[i], bytes));
      HIPCHK(hipEventCreateWithFlags(&c->ev_out[i], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&c->ev_pack[i], hipEventDisableTiming));
    }
  }
  double* dst = c->d_out + (size_t)slot * n * (c->K + 1);
  HIPCHK(hipStreamWaitEvent(c->st, c->ev_out[slot], 0));   // the slot's previous copy
  HIPCHK(launch_pack(c->d_ch, c->nch, c->d_ch_doff, c->xhat1, dst, c->st));
  for (int k = 0; k < c->K; ++k)
    HIPCHK(launch_pack(c->d_ch, c->nch, c->d_ch_doff, c->r1[k], dst + n * (k + 1), c->st));
  // the copy runs on the copy stream: the ctx stream goes on with the step
  HIPCHK(hipEventRecord(c->ev_pack[slot], c->st));
  HIPCHK(hipStreamWaitEvent(c->st_copy, c->ev_pack[slot], 0));
  HIPCHK(hipMemcpyAsync(c->h_out[slot], dst, sizeof(double) * n * (c->K + 1),
                        hipMemcpyDeviceToHost, c->st_copy));
  HIPCHK(hipEventRecord(c->ev_out[slot], c->st_copy));
  return SGV_OK;
}

// May be called from another host thread than the one driving the context: it
// only waits on the slot's event and returns the pinned buffer (valid until the
// slot's next sgv_outputs_begin).
extern "C" int sgv_outputs_wait(sgv_ctx* c, int slot, double** data) {
  if (!c || slot < 0 || slot >= NOUT_SLOTS || !data || !c->ev_out[slot]) return SGV_ERR_ARG;
  if (hipSetDevice(c->dev) != hipSuccess) return SGV_ERR_HIP;
  hipError_t e;
  while ((e = hipEventQuery(c->ev_out[slot])) == hipErrorNotReady) __builtin_ia32_pause();
  if (e != hipSuccess) return SGV_ERR_HIP;
  *data = c->h_out[slot];
  return SGV_OK;
}

extern "C" int sgv_abi_version(void) { return SGV_ABI_VERSION; }

extern "C" int sgv_timers(sgv_ctx* c, double* dst, int cap, int reset) {
  ENTER(c);
  if (cap < 0 || (cap > 0 && !dst)) return fail(c, SGV_ERR_ARG, "sgv_timers: bad buffer");
  CHK(stream_wait(c));
  resolve_timers(c);
  {
    double t6[SGV_TIMERS_N];
    t6[0] = c->ld_ms;
    t6[1] = c->ld_launches;
    t6[2] = c->ld_bytes;
    t6[3] = c->rhs_bytes;
    t6[4] = c->dense_bytes;
    t6[5] = c->aux_bytes;
    t6[6] = c->ld_flops;
    t6[7] = c->ld_flops_wide;
    t6[8] = c->ld_ms_wide;
    t6[9] = c->ld_launches_wide;
    for (int i = 0; i < std::min(cap, SGV_TIMERS_N); ++i) dst[i] = t6[i];
  }
  if (reset) {
    c->ld_ms = c->ld_launches = c->rhs_bytes = c->ld_bytes = c->dense_bytes = c->aux_bytes = 0.0;
    c->ld_flops = c->ld_flops_wide = c->ld_ms_wide = c->ld_launches_wide = 0.0;
  }
  return SGV_OK;
}

extern "C" int sgv_sync(sgv_ctx* c) {
  ENTER(c);
  CHK(stream_wait(c));
  resolve_timers(c);
  return SGV_OK;
}

extern "C" int sgv_read_bw(sgv_ctx* c, int64_t bytes, int reps, double* gbps) {
  ENTER(c);
  const int64_t unit = (int64_t)256 * 1024;
  bytes = bytes / unit * unit;
  if (!gbps || bytes < unit || reps < 1) return fail(c, SGV_ERR_ARG, "sgv_read_bw: bad arguments");
  CHK(stream_wait(c));
  double* buf = nullptr;
  double* out = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = SGV_OK;
  if (hipMalloc(&buf, (size_t)bytes) != hipSuccess || hipMalloc(&out, 256 * sizeof(double)) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    rc = fail(c, SGV_ERR_HIP, "sgv_read_bw: allocation of %.2f GB failed", bytes / 1e9);
  if (rc == SGV_OK && hipMemsetAsync(buf, 0, (size_t)bytes, c->st) != hipSuccess)
    rc = fail(c, SGV_ERR_HIP, "sgv_read_bw: memset failed");
  float best = 0.f;
  for (int r = -1; rc == SGV_OK && r < reps; ++r) {   // r = -1: warm-up
    float ms = 0.f;
    if (hipEventRecord(e0, c->st) != hipSuccess ||
        launch_read_probe(buf, (size_t)bytes, out, c->st) != hipSuccess ||
        hipEventRecord(e1, c->st) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
      rc = fail(c, SGV_ERR_HIP, "sgv_read_bw: probe launch failed");
    else if (r >= 0 && (best == 0.f || ms < best))
      best = ms;
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (buf) (void)hipFree(buf);
  if (out) (void)hipFree(out);
  if (rc != SGV_OK) {
    (void)hipGetLastError();   // clear it: the next launch_* would report this failure
    return rc;
  }
  *gbps = (double)bytes / ((double)best * 1e-3) / 1e9;
  return SGV_OK;
}
