// The cross-rank exchange of libsgvamp_hip.so: every M-length sum is formed per
// LD block and added in global block order, the per-block partials carried by
// an RCCL all-gather (ncclCommInitRank, one process per GPU) or by the host
// exchange callback -- the reference's mpi4py bcast all-gather (src/main.py:16-18,
// src/sgvamp.py:228-233) replaced by ordered sums that leave every scalar
// bitwise independent of the GPU count.  Also the EM prior loop's exchange
// mode (replicated vs per step, a cost model), the latency probe, the counters.
#include "ctx.h"

// every cross-rank all-gather of cnt doubles per rank goes through here: RCCL
// on the ctx stream (timed by events), or the host callback on staged copies
// (timed by the wall clock; the caller's copies are its own)
static int allgather_timed(sgv_ctx* c, const double* d_send, double* d_recv, size_t cnt,
                           const double* h_send, double* h_recv) {
  c->xchg_n += 1.0;
  c->xchg_bytes += 8.0 * (double)cnt;
  if (c->comm) {
    hipEvent_t e0, e1;
    CHK(event_pair(c, &e0, &e1));
    HIPCHK(hipEventRecord(e0, c->st));
    NCCLCHK(ncclAllGather(d_send, d_recv, cnt, ncclDouble, c->comm, c->st));
    HIPCHK(hipEventRecord(e1, c->st));
    c->xpending.emplace_back(e0, e1);
    return SGV_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = c->host_ag(c->host_ag_user, h_send, h_recv, (int64_t)cnt);
  c->xchg_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (rc != 0) return fail(c, SGV_ERR_RCCL, "host all-gather callback failed");
  return SGV_OK;
}

// the exchange half of an ordered reduction: d_bsum [nblk][nv] (this rank's
// per-block sums) -> all ranks' -> d_dst[map.d[v]] in global block order
static int reduce_exchange(sgv_ctx* c, int nv, const Map16& map, double* d_dst, int op) {
  const double* src = c->d_bsum;
  int nr = 1, nbm = c->nblk;
  if (c->comm) {
    CHK(allgather_timed(c, c->d_bsum, c->d_bsum_all, (size_t)c->nbmax * nv, nullptr, nullptr));
  } else if (c->host_ag) {
    const size_t cnt = (size_t)c->nbmax * nv;
    HIPCHK(hipMemcpyAsync(c->h_bsum, c->d_bsum, sizeof(double) * cnt, hipMemcpyDeviceToHost,
                          c->st));
    CHK(stream_wait(c));
    CHK(allgather_timed(c, nullptr, nullptr, cnt, c->h_bsum, c->h_bsum_all));
    HIPCHK(hipMemcpyAsync(c->d_bsum_all, c->h_bsum_all, sizeof(double) * cnt * c->nranks,
                          hipMemcpyHostToDevice, c->st));
  }
  if (c->comm || c->host_ag) {   // [nranks][nbmax][nv] gathered partials, also at one rank
    src = c->d_bsum_all;
    nr = c->nranks;
    nbm = c->nbmax;
  }
  HIPCHK(launch_reduce_total(src, nr, nbm, nv, c->d_counts, map, d_dst, c->st, op));
  return SGV_OK;
}

// partials [nparts][nv] -> d_dst[map.d[v]] (global, ordered); stays on device
int reduce_dev(sgv_ctx* c, int nv, const int* d_begin, const Map16& map, double* d_dst,
                      int op){
  if (!c->comm && !c->host_ag) {   // one rank: fused, bitwise the same as the two steps
    HIPCHK(launch_reduce_local(c->d_part, nv, d_begin, c->nblk, map, d_dst, c->st, op));
    return SGV_OK;
  }
  HIPCHK(launch_reduce_blocks(c->d_part, nv, d_begin, c->nblk, c->d_bsum, c->st, op));
  return reduce_exchange(c, nv, map, d_dst, op);
}

// Two ordered sums in ONE exchange (with a communicator): source A (partials
// partA [part][nvA] over beginA -> d_dst[0 .. nvA)) and the pass partials
// (c->d_part [part][nvB] over beginB -> d_dst[offB + mapB.d[v]]).  Each value
// is the same per-block sums in the same global block order as its own
// reduce_dev: bitwise the two separate reductions.
int reduce_dev2(sgv_ctx* c, const double* partA, int nvA, const int* beginA, int nvB,
                       const int* beginB, const Map16& mapB, int offB, double* d_dst){
  const int nv = nvA + nvB;
  if (nv > MAXNV || (!c->comm && !c->host_ag))
    return fail(c, SGV_ERR_STATE, "reduce_dev2: %d values, or no communicator", nv);
  HIPCHK(launch_reduce_blocks(partA, nvA, beginA, c->nblk, c->d_bsum, c->st, 0, nv, 0));
  HIPCHK(launch_reduce_blocks(c->d_part, nvB, beginB, c->nblk, c->d_bsum, c->st, 0, nv, nvA));
  Map16 m;
  for (int v = 0; v < nvA; ++v) m.d[v] = v;
  for (int v = 0; v < nvB; ++v) m.d[nvA + v] = offB + mapB.d[v];
  return reduce_exchange(c, nv, m, d_dst, 0);
}

// the ordered total is stored by the reduction kernel straight into h_tot
// (fine-grained pinned memory): no copy launch before the host reads it
int reduce_host(sgv_ctx* c, int nv, const int* d_begin, double* out, int op){
  CHK(reduce_dev(c, nv, d_begin, identity_map(), c->h_tot, op));
  CHK(stream_wait(c));
  resolve_timers(c);
  std::memcpy(out, c->h_tot, sizeof(double) * nv);
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// comm
// ---------------------------------------------------------------------------
extern "C" int sgv_comm_unique_id(char* id_out) {
  sgv_ctx* c = nullptr;
  if (!id_out) return fail(nullptr, SGV_ERR_ARG, "id_out is null");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof id);
  return SGV_OK;
}

// buffers of the ordered cross-rank reduction (per-block partials of every rank)
static int comm_buffers(sgv_ctx* c, int nranks, int rank, const int* nblk_per_rank) {
  c->nranks = nranks;
  c->rank = rank;
  c->rank_blk0.assign(nranks + 1, 0);
  for (int r = 0; r < nranks; ++r) c->rank_blk0[r + 1] = c->rank_blk0[r] + nblk_per_rank[r];
  for (auto& p : c->plan) p.valid = false;   // the halo decision depends on the partition
  c->nbmax = *std::max_element(nblk_per_rank, nblk_per_rank + nranks);
  const size_t per = (size_t)c->nbmax * MAXNV;
  HIPCHK(hipFree(c->d_bsum));
  c->d_bsum = nullptr;
  HIPCHK(hipMalloc(&c->d_bsum, sizeof(double) * per));
  HIPCHK(hipMemset(c->d_bsum, 0, sizeof(double) * per));
  HIPCHK(hipMalloc(&c->d_bsum_all, sizeof(double) * per * nranks));
  HIPCHK(hipFree(c->d_counts));
  c->d_counts = nullptr;
  HIPCHK(hipMalloc(&c->d_counts, sizeof(int) * nranks));
  HIPCHK(hipMemcpy(c->d_counts, nblk_per_rank, sizeof(int) * nranks, hipMemcpyHostToDevice));
  return SGV_OK;
}

static int comm_args(sgv_ctx* c, int nranks, int rank, const int* nblk_per_rank) {
  if (nranks < 1 || rank < 0 || rank >= nranks || !nblk_per_rank)
    return fail(c, SGV_ERR_ARG, "bad comm arguments");
  if (nblk_per_rank[rank] != c->nblk)
    return fail(c, SGV_ERR_ARG, "nblk_per_rank[%d]=%d != %d", rank, nblk_per_rank[rank], c->nblk);
  if (c->comm || c->host_ag) return fail(c, SGV_ERR_ARG, "communicator already initialised");
  return SGV_OK;
}

// all-gather of cnt doubles per rank (device buffers), RCCL or the host callback
int gather_f64(sgv_ctx* c, const double* d_send, double* d_recv, size_t cnt,
                      double* h_send, double* h_recv){
  if (c->comm) return allgather_timed(c, d_send, d_recv, cnt, nullptr, nullptr);
  HIPCHK(hipMemcpyAsync(h_send, d_send, sizeof(double) * cnt, hipMemcpyDeviceToHost, c->st));
  CHK(stream_wait(c));
  CHK(allgather_timed(c, nullptr, nullptr, cnt, h_send, h_recv));
  HIPCHK(hipMemcpyAsync(d_recv, h_recv, sizeof(double) * cnt * c->nranks, hipMemcpyHostToDevice,
                        c->st));
  return SGV_OK;
}

// With a communicator the EM prior loop either runs REPLICATED (every rank's r1
// all-gathered once per loop, then the one-rank loop over all M markers on every
// rank -- the reference's own structure, src/sgvamp.py:228-259) or with ONE
// EXCHANGE PER EM STEP (each rank sums its own markers; the per-block partials
// are all-gathered every step, stream-ordered, the loop still device-driven).
// Both give the same bits (ordered per-block sums in global block order), so
// the mode is chosen per EM loop by a cost model whose one machine parameter is
// the per-all-gather latency L (the same value on every rank, so every rank
// picks the same mode):
//   replicated: L + 8 K M (N-1)/N / B + S x (k_em(K M) + T_rep)
//   per step:   S x (k_em(K M / N) + T_ps + L)
// S = the steps the loop enqueues (the predicted EM steps + the one queued
// past the last), predicted as the previous loop's (the first loop: maxit);
// k_em(n) = 5 us + 11 ps per cohort-marker (f64-VALU bound: 44 us at 4e6 on one
// MI355X), T_rep = 35 us (the one-workgroup reduction + control over every
// block), T_ps = 15 us (per-block sums, ordered total, control: 3 launches),
// B = 100 GB/s (an xGMI all-gather of MBs).  L: 25 us by default, env
// SGV_XCHG_LAT_US (rank 0's value), or measured (sgv_exchange_probe).  A
// measured L already holds the per-block sums and ordered-total launches (the
// probe times a whole ordered reduction), so then T_ps keeps only the control
// launch, T_CTL = 5 us (counted once).
// SGV_EM_REP=0/1 (with SGV_AB=1) forces either mode.
constexpr double EM_K_FIX_US = 5.0, EM_K_PER_CM_US = 1.1e-5, EM_T_REP_US = 35.0,
                 EM_T_PS_US = 15.0, EM_T_CTL_US = 5.0, EM_AG_GBS = 100.0;
static void em_costs_raw(double km, double n, double L, double steps, double tps, double* rep_us,
                         double* ps_us) {
  *rep_us = L + 8.0 * km * (n - 1.0) / n / (EM_AG_GBS * 1e3) +
            steps * (EM_K_FIX_US + EM_K_PER_CM_US * km + EM_T_REP_US);
  *ps_us = steps * (EM_K_FIX_US + EM_K_PER_CM_US * km / n + tps + L);
}
static void em_costs(const sgv_ctx* c, double steps, double* rep_us, double* ps_us) {
  em_costs_raw((double)c->K * (double)c->Mtot, (double)c->nranks, c->xlat_us, steps,
               c->xlat_src == 2 ? EM_T_CTL_US : EM_T_PS_US, rep_us, ps_us);
}
// the mode of the next EM loop (maxit steps at most); records the prediction
bool em_mode_pick(sgv_ctx* c, int maxit){
  if (!c->em_rep) return false;
  const double steps = (double)std::min(maxit, (c->em_prev_steps < 0 ? maxit : c->em_prev_steps) + 1);
  em_costs(c, steps, &c->em_pred_rep_us, &c->em_pred_ps_us);
  c->em_pred_steps = steps;
  const char* e = ab_env("SGV_EM_REP");
  const bool rep = e ? e[0] != '0' : c->em_pred_rep_us < c->em_pred_ps_us;
  c->em_last_rep = rep ? 1 : 0;
  (rep ? c->em_loops_rep : c->em_loops_ps) += 1.0;
  return rep;
}

// At communicator set-up: every rank's block sizes and the latency parameter
// (rank 0's) are gathered; then, where the replicated loop can run (K <= MAXK,
// every block within the one-workgroup reduction), the global chunk table and
// the gathered-r1 buffers
static int em_rep_setup(sgv_ctx* c, const int* nblk_per_rank) {
  int nbg = 0;
  for (int r = 0; r < c->nranks; ++r) nbg += nblk_per_rank[r];
  const size_t nb = (size_t)c->nbmax + 1;   // [block sizes..., latency]
  double *d_s = nullptr, *d_r = nullptr;
  std::vector<double> hs(nb, 0.0), hr(nb * c->nranks, 0.0);
  for (int b = 0; b < c->nblk; ++b) hs[b] = (double)c->bn[b];
  {
    const char* e = std::getenv("SGV_XCHG_LAT_US");
    char* end = nullptr;
    const double v = (e && *e) ? std::strtod(e, &end) : -1.0;
    hs[nb - 1] = (e && end != e && v >= 0.0) ? v : -1.0;
  }
  double *h_s = nullptr, *h_r = nullptr;
  int rc = SGV_OK;
  if (hipMalloc(&d_s, sizeof(double) * nb) != hipSuccess ||
      hipMalloc(&d_r, sizeof(double) * nb * c->nranks) != hipSuccess ||
      hipHostMalloc(&h_s, sizeof(double) * nb) != hipSuccess ||
      hipHostMalloc(&h_r, sizeof(double) * nb * c->nranks) != hipSuccess)
    rc = fail(c, SGV_ERR_HIP, "em_rep_setup: allocation failed");
  if (rc == SGV_OK && hipMemcpy(d_s, hs.data(), sizeof(double) * nb, hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(c, SGV_ERR_HIP, "em_rep_setup: copy failed");
  if (rc == SGV_OK) rc = gather_f64(c, d_s, d_r, nb, h_s, h_r);
  if (rc == SGV_OK && hipStreamSynchronize(c->st) != hipSuccess)
    rc = fail(c, SGV_ERR_HIP, "em_rep_setup: sync failed");
  if (rc == SGV_OK && hipMemcpy(hr.data(), d_r, sizeof(double) * nb * c->nranks, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(c, SGV_ERR_HIP, "em_rep_setup: copy failed");
  if (d_s) (void)hipFree(d_s);
  if (d_r) (void)hipFree(d_r);
  if (h_s) (void)hipHostFree(h_s);
  if (h_r) (void)hipHostFree(h_r);
  CHK(rc);
  if (hr[nb - 1] >= 0.0) {   // rank 0's SGV_XCHG_LAT_US
    c->xlat_us = hr[nb - 1];
    c->xlat_src = 1;
  }
  if (c->K > MAXK || nbg > EM_CTL_MAXBLK) return SGV_OK;   // per-step exchange only
  // per-rank padded layouts (the rule of sgv_create), then the global chunks
  std::vector<std::vector<int64_t>> bv(c->nranks);
  int64_t mpmax = PADV;
  for (int r = 0; r < c->nranks; ++r) {
    int64_t v = 0;
    for (int b = 0; b < nblk_per_rank[r]; ++b) {
      const int64_t n = (int64_t)hr[(size_t)r * nb + b];
      if (n < 1) return fail(c, SGV_ERR_ARG, "em_rep_setup: rank %d block %d size %lld", r, b,
                             (long long)n);
      bv[r].push_back(v);
      v += round_up(n, PADV);
    }
    mpmax = std::max(mpmax, std::max<int64_t>(v, PADV));
  }
  if (c->Mpad > mpmax) return fail(c, SGV_ERR_ARG, "em_rep_setup: inconsistent layouts");
  std::vector<ChunkDesc> ch;
  std::vector<int> chb;
  int gb = 0;
  for (int r = 0; r < c->nranks; ++r)
    for (int b = 0; b < nblk_per_rank[r]; ++b, ++gb) {
      chb.push_back((int)ch.size());
      const int64_t n = (int64_t)hr[(size_t)r * nb + b];
      const int64_t base = (int64_t)r * c->K * mpmax + bv[r][b];
      for (int64_t o = 0; o < n; o += CHUNK)
        ch.push_back(ChunkDesc{base + o, (int32_t)std::min<int64_t>(CHUNK, n - o), gb});
    }
  chb.push_back((int)ch.size());
  c->mpad_max = mpmax;
  c->nchg = (int)ch.size();
  c->nblkg = gb;
  HIPCHK(hipMalloc(&c->d_chg, sizeof(ChunkDesc) * ch.size()));
  HIPCHK(hipMemcpy(c->d_chg, ch.data(), sizeof(ChunkDesc) * ch.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&c->d_chg_begin, sizeof(int) * chb.size()));
  HIPCHK(hipMemcpy(c->d_chg_begin, chb.data(), sizeof(int) * chb.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&c->d_partg, sizeof(double) * ch.size() * EM_NV));
  const size_t per = (size_t)c->K * mpmax;
  HIPCHK(hipMalloc(&c->d_r1send, sizeof(double) * per));
  HIPCHK(hipMemset(c->d_r1send, 0, sizeof(double) * per));
  HIPCHK(hipMalloc(&c->d_r1g, sizeof(double) * per * c->nranks));
  if (!c->comm) {
    HIPCHK(hipHostMalloc(&c->h_r1send, sizeof(double) * per));
    HIPCHK(hipHostMalloc(&c->h_r1g, sizeof(double) * per * c->nranks));
  }
  c->em_rep = true;
  return SGV_OK;
}

// every cohort's r1 from every rank -> d_r1g (once per EM loop)
int gather_r1(sgv_ctx* c){
  for (int k = 0; k < c->K; ++k)
    HIPCHK(hipMemcpyAsync(c->d_r1send + (size_t)k * c->mpad_max, c->r1[k],
                          sizeof(double) * c->Mpad, hipMemcpyDeviceToDevice, c->st));
  return gather_f64(c, c->d_r1send, c->d_r1g, (size_t)c->K * c->mpad_max, c->h_r1send, c->h_r1g);
}

extern "C" int sgv_comm_init(sgv_ctx* c, int nranks, int rank, const char* id,
                             const int* nblk_per_rank) {
  ENTER(c);
  if (!id) return fail(c, SGV_ERR_ARG, "bad comm arguments");
  CHK(comm_args(c, nranks, rank, nblk_per_rank));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  NCCLCHK(ncclCommInitRank(&c->comm, nranks, uid, rank));
  CHK(comm_buffers(c, nranks, rank, nblk_per_rank));
  return em_rep_setup(c, nblk_per_rank);
}

extern "C" int sgv_comm_init_host(sgv_ctx* c, int nranks, int rank, const int* nblk_per_rank,
                                  sgv_allgather_fn fn, void* user) {
  ENTER(c);
  if (!fn) return fail(c, SGV_ERR_ARG, "allgather callback is null");
  CHK(comm_args(c, nranks, rank, nblk_per_rank));
  CHK(comm_buffers(c, nranks, rank, nblk_per_rank));
  const size_t per = (size_t)c->nbmax * MAXNV;
  HIPCHK(hipHostMalloc(&c->h_bsum, sizeof(double) * per));
  HIPCHK(hipHostMalloc(&c->h_bsum_all, sizeof(double) * per * nranks));
  c->host_ag = fn;
  c->host_ag_user = user;
  return em_rep_setup(c, nblk_per_rank);
}

extern "C" int sgv_exchange_stats(sgv_ctx* c, double* dst, int cap, int reset) {
  ENTER(c);
  if (cap < 0 || (cap > 0 && !dst)) return fail(c, SGV_ERR_ARG, "sgv_exchange_stats: bad buffer");
  CHK(stream_wait(c));
  resolve_timers(c);
  const bool cm = c->comm || c->host_ag;
  double out[SGV_EXCHANGE_STATS_N];
  out[0] = c->xchg_n;
  out[1] = c->xchg_ms;
  out[2] = c->xchg_bytes;
  out[3] = cm ? (double)c->em_last_rep : -1.0;
  out[4] = c->xlat_us;
  out[5] = c->comm ? 1.0 : c->host_ag ? 2.0 : 0.0;
  out[6] = c->em_loops_rep;
  out[7] = c->em_loops_ps;
  out[8] = cm ? c->em_pred_rep_us : 0.0;
  out[9] = cm ? c->em_pred_ps_us : 0.0;
  out[10] = c->em_pred_steps;
  out[11] = c->host_wait_ms;
  out[12] = (double)c->xlat_src;
  out[13] = c->em_rep ? 1.0 : 0.0;
  out[14] = c->em_ms;
  out[15] = c->em_loops_timed;
  for (int i = 0; i < std::min(cap, SGV_EXCHANGE_STATS_N); ++i) dst[i] = out[i];
  if (reset) {
    c->xchg_n = c->xchg_ms = c->xchg_bytes = 0.0;
    c->em_loops_rep = c->em_loops_ps = 0.0;
    c->host_wait_ms = 0.0;
    c->em_ms = c->em_loops_timed = 0.0;
  }
  return SGV_OK;
}

extern "C" int sgv_comm_info(sgv_ctx* c, int* dst, int cap, char* pci_bus_id, int pci_len) {
  ENTER(c);
  if (cap < 0 || (cap > 0 && !dst) || (pci_bus_id && pci_len < 1))
    return fail(c, SGV_ERR_ARG, "sgv_comm_info: bad buffer");
  int out[SGV_COMM_INFO_N] = {c->comm ? 1 : c->host_ag ? 2 : 0, c->nranks, c->rank, c->dev,
                              c->nranks};
  if (c->comm) {
    NCCLCHK(ncclCommCount(c->comm, &out[1]));
    NCCLCHK(ncclCommUserRank(c->comm, &out[2]));
    NCCLCHK(ncclCommCuDevice(c->comm, &out[3]));
  } else if (!c->host_ag) {
    out[1] = 1;
    out[2] = 0;
  }
  for (int i = 0; i < std::min(cap, SGV_COMM_INFO_N); ++i) dst[i] = out[i];
  if (pci_bus_id) HIPCHK(hipDeviceGetPCIBusId(pci_bus_id, pci_len, out[3]));
  return SGV_OK;
}

// The per-all-gather latency of this job's exchange, measured: `reps` ordered
// reductions of MAXC values over the per-block partials (the CG's own exchange:
// per-block sums, all-gather, ordered total) on the ctx stream, after one
// untimed; RCCL: HIP events around them (the wait for the slowest peer
// included), host exchange: wall time.  The maximum over ranks becomes the EM
// cost model's L on every rank (em_costs).  Collective: every rank calls it,
// between steps.  *us_out = the agreed latency (0 without a communicator).
extern "C" int sgv_exchange_probe(sgv_ctx* c, int reps, double* us_out) {
  ENTER(c);
  if (!us_out || reps < 1) return fail(c, SGV_ERR_ARG, "sgv_exchange_probe: bad arguments");
  *us_out = 0.0;
  if (!c->comm && !c->host_ag) return SGV_OK;
  CHK(stream_wait(c));
  resolve_timers(c);
  const double n0 = c->xchg_n, ms0 = c->xchg_ms, b0 = c->xchg_bytes;
  CHK(reduce_dev(c, MAXC, c->d_ch_begin, identity_map(), c->d_tot));   // untimed
  CHK(stream_wait(c));
  hipEvent_t e0, e1;
  CHK(event_pair(c, &e0, &e1));
  const auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipEventRecord(e0, c->st));
  for (int r = 0; r < reps; ++r) CHK(reduce_dev(c, MAXC, c->d_ch_begin, identity_map(), c->d_tot));
  HIPCHK(hipEventRecord(e1, c->st));
  CHK(stream_wait(c));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  c->evpool.push_back(e0);
  c->evpool.push_back(e1);
  const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const double us = 1e3 * (c->comm ? (double)ms : wall) / reps;
  // agree: every rank's value, the maximum
  CHK(ensure_stage(c, sizeof(double) * (1 + (size_t)c->nranks)));
  CHK(ensure_hstage(c, sizeof(double) * (1 + (size_t)c->nranks)));
  double* hs = (double*)c->h_stage;
  double* ds = (double*)c->d_stage;
  hs[0] = us;
  HIPCHK(hipMemcpyAsync(ds, hs, sizeof(double), hipMemcpyHostToDevice, c->st));
  CHK(gather_f64(c, ds, ds + 1, 1, hs, hs + 1));
  HIPCHK(hipMemcpyAsync(hs + 1, ds + 1, sizeof(double) * c->nranks, hipMemcpyDeviceToHost, c->st));
  CHK(stream_wait(c));
  resolve_timers(c);
  double agreed = 0.0;
  for (int r = 0; r < c->nranks; ++r) agreed = std::max(agreed, hs[1 + r]);
  c->xlat_us = agreed;
  c->xlat_src = 2;
  c->xchg_n = n0;   // the probe is not the job's exchange
  c->xchg_ms = ms0;
  c->xchg_bytes = b0;
  *us_out = agreed;
  return SGV_OK;
}

extern "C" int sgv_em_cost_model(double cohort_markers, int nranks, double latency_us,
                                 double steps, double* out2) {
  if (!out2 || nranks < 1 || !(cohort_markers >= 0.0) || !(latency_us >= 0.0) || !(steps >= 0.0))
    return SGV_ERR_ARG;
  em_costs_raw(cohort_markers, (double)nranks, latency_us, steps, EM_T_PS_US, &out2[0], &out2[1]);
  return SGV_OK;
}
