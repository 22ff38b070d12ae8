// C ABI of libsgvamp_hip.so (declared in include/sgvamp_hip.h).
//
// Owns device memory, the HIP stream, the RCCL communicator and the host-side
// drivers of the hot path: the batched scipy-1.15.3 CG loop (one LD pass per CG
// iteration serves every right-hand side still iterating), the LMMSE step,
// the denoiser and the EM prior loop.  Scalar bookkeeping mirrors the
// reference expressions (src/sgvamp.py cited per line); all vector arithmetic
// runs in the HIP kernels of ld_pass.hip / vec.hip / synth.hip.
#include "common.h"
#include "hybrd.h"
#include "../../include/sgvamp_hip.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <limits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

using namespace sgv;

static thread_local std::string g_last_err;

// one LD block of one LD matrix
struct LdBlock {
  double* ptr = nullptr;
  int fmt = 0;                 // 0: dense n x lda row-major; 1: packed symmetric panels
  // packed band: panel g stores columns r0 .. r0 + min(n - r0, ext) - 1 only
  // (ext a multiple of BAND_Q; 0 = the whole upper triangle)
  int64_t ext = 0;
  std::vector<int64_t> poff, pw;   // packed: panel offsets and row strides (doubles)
  int64_t* d_poff = nullptr;
  int64_t* d_pw = nullptr;
  double stored_bytes = 0.0;   // bytes a pass reads: n^2*8 dense, sum H_g (n - r0_g)*8 packed
};

// coupling between consecutive band pieces gb and gb + 1 of one LD matrix (a
// band block too long for one GPU, cut into pieces that ranks can own):
// C = R[last nr rows of gb][first nc columns of gb + 1], kept by the ranks that
// own either piece (sgv_set_ld_coupling)
struct LdCoupling {
  int gb = -1, nr = 0, nc = 0;
  double* d_up = nullptr;   // C^T (nc x nr): side 0, on gb's rank
  double* d_lo = nullptr;   // C (nr x nc): side 1, on gb + 1's rank
};

// launch tables of one LD matrix (rebuilt when a block's storage changes)
struct LdPlan {
  bool valid = false;
  RowGroup* d_rg = nullptr;    // dense blocks
  int nrg = 0;
  int* d_pbeg = nullptr;       // partial slots of block b: [pbeg[b], pbeg[b+1])
  int nparts = 0;
  SymItem* d_items[4] = {nullptr, nullptr, nullptr, nullptr};   // per chunk width class
  int nitems[4] = {0, 0, 0, 0};
  SymPanel* d_panels[4] = {nullptr, nullptr, nullptr, nullptr};
  int npanels = 0;
  // MFMA pass: strips (dispatch order), their class-1 items in strip order, and
  // the class-1 panels with their strip ranges
  SymStrip* d_strips = nullptr;
  SymItem* d_sitems = nullptr;
  SymPanel* d_spanels = nullptr;
  int nstrips = 0;
  bool ragged = false;         // some strip item is narrower than its strip (band blocks)
  int pair = 0;                // k_sym_mfma_pair for 3-4 columns (1) / 3-8 (2) (build_strips)
  // block groups of the MFMA pass (contiguous blocks): group g's strips are
  // d_strips[gs[g] .. gs[g+1]), its panels d_spanels[gp[g] .. gp[g+1]) -- group
  // g's finalize runs on the side stream while group g + 1's strips run
  int ngrp = 1;
  std::vector<int> gs, gp;
  double stored_bytes = 0.0, dense_bytes = 0.0;
  // coupled band pieces: k_coupling tasks, panel slots of PassArgs::cpbuf, and
  // the halo this rank sends (head of its first block, tail of its last) when a
  // coupling spans two ranks -- the same decision on every rank (all ranks know
  // every coupling and the block partition)
  CouplingTask* d_ctasks = nullptr;
  int nctasks = 0, ncp = 0;
  bool halo = false;
  int64_t hmax = 0, h_src0 = 0, h_src1 = 0;
  int h_len0 = 0, h_len1 = 0;
  double cpl_bytes = 0.0;      // coupling matrix bytes read per pass (this rank)
};

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

// chunk-width class of the packed VALU pass for nc columns (CW = 1024 >> cls)
static int sym_class(int nc) { return nc <= 2 ? 0 : nc <= 4 ? 1 : nc <= 8 ? 2 : 3; }
// default number of right-hand sides from which packed passes run on the f64
// matrix cores (sym_mfma.hip, class-1 items); env SGV_MFMA_MIN overrides,
// 0 disables; per context: sgv_set_mfma_min
static int mfma_min_default() {
  static const int v = [] {
    const char* e = ab_env("SGV_MFMA_MIN");
    return e ? std::atoi(e) : 3;
  }();
  return v;
}
// CG loop driver: 1 (default) = pipelined, device-side control (cg_loop_dev);
// 0 = host-side stop test per iteration (cg_loop).  Env SGV_CG_PIPE.
static int cg_pipe_default() {
  const char* e = ab_env("SGV_CG_PIPE");
  return (e && e[0] == '0') ? 0 : 1;
}
constexpr int CG_RING = 4;   // mirror slots of the pipelined CG
constexpr int MAXGRP = 8;    // block groups of one MFMA pass (pass_groups)
constexpr int NOUT_SLOTS = 3;   // pinned output slots (a writer reads one while two steps run)

// SGV_CG_EXACT=0: the pipelined CG's pass of iteration it also carries the
// columns that stop at it's own test (one iteration of look-ahead; A/B);
// sgv_set_cg_exact sets the run's mode (the Engine: from the global LD size)
static int cg_exact_default() {   // -1: by size (cg_loop_dev); 0 / 1 forced (A/B)
  const char* e = ab_env("SGV_CG_EXACT");
  return !e ? -1 : (e[0] == '0' ? 0 : 1);
}
// exact CG column sets by size: a pass narrowed from 8 to 4 columns saves ~4 %
// of its time (north star in the solver: 10.6-10.9 vs 11.0-11.5 ms) against
// ~30 us of host read per CG iteration, so only passes of >= ~4 ms (24 GB
// stored) narrow.  The choice must be the same on every rank and for every
// rank count (the modes can round differently): with a communicator the
// default (-1) is look-ahead, and the Engine sets the mode from the global size
constexpr double CG_EXACT_MIN_BYTES = 24e9;
static int sym_class_nc(int cls) { return std::min(16, 2 << (cls + 1)); }   // widest NC using cls

// The one-workgroup reduction + control kernels (k_cg_reduce_ctl,
// k_em_reduce_ctl) walk nv x nblk (value, block) pairs 128 at a time, each round
// a chain of dependent loads; above one round the two-launch form (k_reduce_local
// over nv workgroups, then the one-wave control kernel; the same bits) is
// faster: at 64 blocks 58 / 40 us fused vs ~9 + 5 us (north-star trace).
static bool fused_ctl_pays(int nv, int nblk) {
  return nblk <= EM_CTL_MAXBLK && nv * nblk <= 128;
}

struct sgv_ctx {
  int dev = 0;
  hipStream_t st = nullptr;
  int K = 0, nld = 0;
  std::vector<int> ld_of;
  // marker partition
  int nblk = 0;
  std::vector<int64_t> bn, boff, bvoff;
  int64_t Mloc = 0, Mpad = 0;
  int blk0 = 0, nblk_global = 0;
  int64_t Mtot = 0;
  double s = 0.0;
  std::vector<double> Ncoh;
  // LD storage [ld][b] and the per-LD launch plans
  std::vector<std::vector<LdBlock>> ldb;
  std::vector<int64_t> lda;
  std::vector<BlkDesc*> d_blks;
  std::vector<LdPlan> plan;
  std::vector<std::vector<LdCoupling>> cpl;   // [ld]: couplings of band pieces
  std::vector<int> rank_blk0;    // first global block of each rank, then nblk_global
  double* d_cpbuf = nullptr;     // coupling sums [slot][256][nc]
  size_t cpbuf_cap = 0;
  double* d_halo = nullptr;      // send [2][nc][hmax] then receive [nranks][2][nc][hmax]
  size_t halo_cap = 0;
  double* h_halo = nullptr;      // pinned staging of the host exchange (same layout)
  size_t h_halo_cap = 0;
  int packing = 1;               // 1: packed symmetric storage for symmetric blocks
  // MFMA passes in block groups (LdPlan::ngrp): the finalize of each group on
  // st_fin behind its strips' event, joined back into st at the pass end
  hipStream_t st_fin = nullptr;
  hipEvent_t ev_grp[MAXGRP] = {};
  hipEvent_t ev_fin = nullptr;
  double* d_rowpart = nullptr;   // k_sym_pass row partials
  double* d_colpart = nullptr;   // k_sym_pass column partials
  size_t rowpart_cap = 0, colpart_cap = 0, part_cap = 0;
  int mfma_min = 3;              // see mfma_min_default
  double* d_pk = nullptr;        // RHS interleaved [Mpad][16] for the MFMA pass
  // asynchronous per-iteration outputs (xhat1, r1[k]): device pack buffer and two
  // pinned host slots, each with its completion event (sgv_outputs_begin/wait)
  double* d_out = nullptr;
  double* h_out[NOUT_SLOTS] = {};
  hipEvent_t ev_out[NOUT_SLOTS] = {};
  // probe upload: two pinned slots used alternately, stream-ordered copy into
  // d_probe (no host wait; a slot is reused two iterations later)
  int8_t* h_probe[2] = {nullptr, nullptr};
  hipEvent_t ev_probe[2] = {nullptr, nullptr};
  int8_t* d_probe = nullptr;
  std::atomic<size_t> probe_cap{0};            // stored after the buffers (read by sgv_step_begin)
  std::atomic<int> probe_slot{0};             // next slot (sgv_step_begin stages from the caller's thread)
  hipEvent_t ev_unpk[2] = {nullptr, nullptr};   // the slot's probes consumed (ctx stream)
  int pref_slot = -1;                           // probes prefetched by sgv_step
  const int8_t* pref_src = nullptr;
  // copies between host and device run on their own stream, behind events: a
  // DMA copy queued on the ctx stream stalls the kernels behind it for its
  // start-up latency (~50-110 us measured per copy)
  hipStream_t st_copy = nullptr;
  hipEvent_t ev_pack[NOUT_SLOTS] = {};
  // metrics queued behind the denoiser, read at the end of the iteration
  double* h_met = nullptr;        // fine-grained pinned [4]
  hipEvent_t ev_met = nullptr;
  int met_pending = 0;
  // sgv_step_begin/end: one host worker thread runs queued steps
  std::thread worker;
  std::mutex wmu;
  std::condition_variable wcv;
  struct Job {
    std::function<int()> fn;
    std::atomic<int> state{0};   // 0 free, 1 queued, 2 running, 3 done
    int rc = 0;
  };
  Job jobs[2];                   // at most two steps in flight, run in order
  uint64_t job_begun = 0, job_ended = 0, job_run = 0;
  std::atomic<bool> worker_quit{false};
  // the last completed sgv_step's results, the inputs of a chained step
  struct Chain {
    int valid = 0;
    std::vector<double> gam1, gamw, alpha1, alpha2;   // K each (sgv_create)
    double lam, om[MAXL];
  } chain;
  // the MLE prior update's Lagrange multiplier (src/sgvamp.py:31,194,211; NaN = None)
  double mle_gam = std::numeric_limits<double>::quiet_NaN();
  double* d_inner = nullptr;      // K > MAXK: the denoiser's np.inner over all cohorts
  size_t inner_cap = 0;
  size_t pk_cap = 0;
  // chunk / row-group layouts
  int nch = 0;
  ChunkDesc* d_ch = nullptr;
  int64_t* d_ch_doff = nullptr;
  int* d_ch_begin = nullptr;
  // vectors (padded layout, zero padding)
  double* pool = nullptr;
  std::vector<double*> r, r1, r2, U, X, X0, Rr, P, Q, RX0, Y, RXp, S;
  double* xhat1 = nullptr;
  double* x0 = nullptr;
  // reductions
  double* d_part = nullptr;
  double* d_part2 = nullptr;    // the LMMSE init's partials when they share an exchange
  size_t part2_cap = 0;
  double* d_bsum = nullptr;
  double* d_bsum_all = nullptr;
  int* d_counts = nullptr;
  double* d_tot = nullptr;
  double* h_tot = nullptr;
  double* d_pq = nullptr;
  int nbmax = 0;
  // staging (device) and pinned host staging: every host<->device copy goes
  // through pinned memory and a spin wait (pageable copies block inside the
  // runtime with its default wait policy)
  void* d_stage = nullptr;
  size_t stage_bytes = 0;
  void* h_stage = nullptr;
  size_t h_stage_bytes = 0;
  // comm
  ncclComm_t comm = nullptr;
  sgv_allgather_fn host_ag = nullptr;   // host exchange (sgv_comm_init_host)
  void* host_ag_user = nullptr;
  double* h_bsum = nullptr;             // pinned [nbmax * MAXNV] and [nranks][nbmax * MAXNV]
  double* h_bsum_all = nullptr;
  int nranks = 1, rank = 0;
  // solver state
  std::vector<int> xnz;        // x0.any() per CG column (2K)
  std::vector<int> rx0_valid;  // RX0[c] == R_s X[c]
  int rs_rec = 1;              // carry R_s x through the CG (sgv_set_rs_recurrence)
  hipEvent_t ev_sync = nullptr;   // host waits spin on this event
  // pipelined CG (cg_loop_dev): device control state, its host mirror ring
  // (fine-grained pinned, one slot per in-flight iteration), init staging
  int cg_pipe = 1;
  int cg_exact = -1;  // pipelined CG: passes carry only the columns active after their test
                      // (-1: by size, cg_loop_dev)
  CgState* d_cgs = nullptr;
  CgState* h_cgm = nullptr;       // [CG_RING]
  CgState* h_cgi = nullptr;
  double* d_rhonew = nullptr;
  hipEvent_t ev_cg[4] = {nullptr, nullptr, nullptr, nullptr};
  // device EM loop (sgv_em with cg_pipe on): state, mirror ring, init staging
  EmState* d_ems = nullptr;
  // replicated EM (with a communicator): every rank's r1 is all-gathered once per
  // EM loop and the loop runs over all markers on every rank with one-rank
  // reductions -- the reference's r1 all-gather + redundant EM (sgvamp.py:228-259)
  // instead of one exchange per EM step.  Global chunk table in global block
  // order (the same sums as one rank); gathered r1 as [nranks][K][mpad_max].
  bool em_rep = false;          // the replicated loop's buffers are set up (em_rep_setup)
  // EM exchange cost model (em_mode_pick): the per-all-gather latency in force
  // (us; the same on every rank: rank 0's at set-up, or the probe's maximum over
  // ranks), its source (0 default, 1 env SGV_XCHG_LAT_US, 2 measured by
  // sgv_exchange_probe), the steps of the last EM loop (the next one's
  // prediction), the last decision's predicted costs and the loops per mode
  double xlat_us = 25.0;
  int xlat_src = 0;
  int em_prev_steps = -1;
  int em_last_rep = -1;
  double em_pred_rep_us = 0.0, em_pred_ps_us = 0.0, em_pred_steps = 0.0;
  double em_loops_rep = 0.0, em_loops_ps = 0.0;
  // exact CG column sets: host time spent waiting for a stop test before the
  // passes can be enqueued (the device bubble's upper bound)
  double host_wait_ms = 0.0;
  int nchg = 0, nblkg = 0;
  int64_t mpad_max = 0;
  ChunkDesc* d_chg = nullptr;
  int* d_chg_begin = nullptr;
  double* d_partg = nullptr;
  double* d_r1send = nullptr;   // [K][mpad_max]
  double* d_r1g = nullptr;      // [nranks][K][mpad_max]
  double* h_r1send = nullptr;   // host exchange staging
  double* h_r1g = nullptr;
  EmState* h_emm = nullptr;       // [CG_RING]
  EmState* h_emi = nullptr;
  double* d_emtot = nullptr;
  double* d_emtab = nullptr;      // [K][EM_TAB] per-cohort EM constants (k_em_prep)
  hipEvent_t ev_em[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_den = nullptr;    // sgv_step: the denoiser's sums are in h_tot
  // timers
  std::vector<hipEvent_t> evpool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  // cross-rank exchange counters (sgv_exchange_stats): all-gathers issued, the
  // bytes each rank contributed, and their time -- HIP events around every
  // ncclAllGather on the ctx stream (the wait for the slowest peer included),
  // wall time of the host callback for the host exchange
  std::vector<std::pair<hipEvent_t, hipEvent_t>> xpending;
  double xchg_n = 0.0, xchg_ms = 0.0, xchg_bytes = 0.0;
  double ld_ms = 0.0, ld_launches = 0.0, rhs_bytes = 0.0, ld_bytes = 0.0, dense_bytes = 0.0,
         aux_bytes = 0.0;
  std::string err;
};

// ---------------------------------------------------------------------------
// error handling
// ---------------------------------------------------------------------------
static int fail(sgv_ctx* c, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  g_last_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(c, SGV_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                              \
  } while (0)

#define NCCLCHK(expr)                                                                     \
  do {                                                                                    \
    ncclResult_t e_ = (expr);                                                             \
    if (e_ != ncclSuccess)                                                                \
      return fail(c, SGV_ERR_RCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(e_),        \
                  __FILE__, __LINE__);                                                    \
  } while (0)

#define CHK(expr)               \
  do {                          \
    int rc_ = (expr);           \
    if (rc_ != SGV_OK) return rc_; \
  } while (0)

#define ENTER(c)                                                   \
  do {                                                             \
    if (!(c)) return fail(nullptr, SGV_ERR_ARG, "null context");   \
    HIPCHK(hipSetDevice((c)->dev));                                \
  } while (0)

static int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Host wait for the ctx stream: record an event and spin on it.  The default
// hipStreamSynchronize may park the thread and wake it late (measured on
// MI355X: ~10 ms extra per wait), and the CG loop waits once per iteration.
static int stream_wait(sgv_ctx* c) {
  HIPCHK(hipEventRecord(c->ev_sync, c->st));
  hipError_t e;
  while ((e = hipEventQuery(c->ev_sync)) == hipErrorNotReady) {
    __builtin_ia32_pause();
  }
  if (e != hipSuccess)
    return fail(c, SGV_ERR_HIP, "stream wait: %s", hipGetErrorString(e));
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------
static Map16 identity_map() {
  Map16 m;
  for (int i = 0; i < MAXNV; ++i) m.d[i] = i;
  return m;
}

static void resolve_timers(sgv_ctx* c) {
  for (auto& pr : c->pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) c->ld_ms += ms;
    c->evpool.push_back(pr.first);
    c->evpool.push_back(pr.second);
  }
  c->pending.clear();
  for (auto& pr : c->xpending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) c->xchg_ms += ms;
    c->evpool.push_back(pr.first);
    c->evpool.push_back(pr.second);
  }
  c->xpending.clear();
}

static int event_pair(sgv_ctx* c, hipEvent_t* e0, hipEvent_t* e1) {
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
static int reduce_dev(sgv_ctx* c, int nv, const int* d_begin, const Map16& map, double* d_dst,
                      int op = 0) {
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
static int reduce_dev2(sgv_ctx* c, const double* partA, int nvA, const int* beginA, int nvB,
                       const int* beginB, const Map16& mapB, int offB, double* d_dst) {
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
static int reduce_host(sgv_ctx* c, int nv, const int* d_begin, double* out, int op = 0) {
  CHK(reduce_dev(c, nv, d_begin, identity_map(), c->h_tot, op));
  CHK(stream_wait(c));
  resolve_timers(c);
  std::memcpy(out, c->h_tot, sizeof(double) * nv);
  return SGV_OK;
}

static int ensure_stage(sgv_ctx* c, size_t bytes) {
  if (bytes <= c->stage_bytes) return SGV_OK;
  if (c->d_stage) HIPCHK(hipFree(c->d_stage));
  c->d_stage = nullptr;
  HIPCHK(hipMalloc(&c->d_stage, bytes));
  c->stage_bytes = bytes;
  return SGV_OK;
}

static int ensure_hstage(sgv_ctx* c, size_t bytes) {
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
static int probe_stage(sgv_ctx* c, const int8_t* probes) {
  const int slot = c->probe_slot.fetch_xor(1);
  if (hipEventSynchronize(c->ev_probe[slot]) != hipSuccess) {
    fail(c, SGV_ERR_HIP, "probe slot wait failed");
    return -1;
  }
  std::memcpy(c->h_probe[slot], probes, (size_t)c->K * c->Mloc);
  return slot;
}
static int probe_issue(sgv_ctx* c, int slot, int* slot_out);

// K x Mloc int8 probes -> d_probe slot, copied on the copy stream (no host wait);
// returns the slot.  A slot's device half is consumed by the unpack kernels of
// its step (ev_unpk) and reused two uploads later.
static int probe_upload(sgv_ctx* c, const int8_t* probes, int* slot_out) {
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
static int probe_issue(sgv_ctx* c, int slot, int* slot_out) {
  HIPCHK(hipStreamWaitEvent(c->st_copy, c->ev_unpk[slot], 0));
  HIPCHK(hipMemcpyAsync(c->d_probe + slot * c->probe_cap, c->h_probe[slot],
                        (size_t)c->K * c->Mloc, hipMemcpyHostToDevice, c->st_copy));
  HIPCHK(hipEventRecord(c->ev_probe[slot], c->st_copy));
  *slot_out = slot;
  return SGV_OK;
}

static int upload_vec(sgv_ctx* c, const double* host, double* dpad) {
  CHK(h2d(c, host, sizeof(double) * c->Mloc));
  HIPCHK(launch_unpack(c->d_ch, c->nch, c->d_ch_doff, (const double*)c->d_stage, dpad, c->st));
  return SGV_OK;
}

static int download_vec(sgv_ctx* c, const double* dpad, double* host) {
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

static bool host_any(const double* v, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    if (v[i] != 0.0) return true;
  return false;
}

// ---------------------------------------------------------------------------
// LD pass (timed with HIP events on the ctx stream)
// ---------------------------------------------------------------------------
static void free_plan(LdPlan& p) {
  if (p.d_rg) (void)hipFree(p.d_rg);
  if (p.d_pbeg) (void)hipFree(p.d_pbeg);
  for (int k = 0; k < 4; ++k) {
    if (p.d_items[k]) (void)hipFree(p.d_items[k]);
    if (p.d_panels[k]) (void)hipFree(p.d_panels[k]);
  }
  if (p.d_strips) (void)hipFree(p.d_strips);
  if (p.d_sitems) (void)hipFree(p.d_sitems);
  if (p.d_spanels) (void)hipFree(p.d_spanels);
  if (p.d_ctasks) (void)hipFree(p.d_ctasks);
  p = LdPlan();
}

static void free_block(LdBlock& lb) {
  if (lb.ptr) (void)hipFree(lb.ptr);
  if (lb.d_poff) (void)hipFree(lb.d_poff);
  if (lb.d_pw) (void)hipFree(lb.d_pw);
  lb = LdBlock();
}

// stored columns of panel g (first row r0) of an n-row packed block
static int64_t panel_ext(int64_t n, int64_t r0, int64_t ext) {
  return ext > 0 ? std::min(n - r0, ext) : n - r0;
}

// allocate block b of LD matrix ld in format fmt (zero filled); ext: packed
// band extent (0 = full upper triangle)
static int ld_alloc(sgv_ctx* c, int ld, int b, int fmt, int64_t ext = 0) {
  LdBlock& lb = c->ldb[ld][b];
  if (fmt == 0) ext = 0;
  if (lb.ptr && lb.fmt == fmt && lb.ext == ext) return SGV_OK;
  free_block(lb);
  c->plan[ld].valid = false;
  const int64_t n = c->bn[b];
  size_t elems = 0;
  lb.fmt = fmt;
  lb.ext = ext;
  if (fmt == 0) {
    elems = (size_t)c->lda[b] * (size_t)n;
    lb.stored_bytes = (double)n * (double)n * 8.0;
  } else {
    double valid = 0.0;
    for (int64_t r0 = 0; r0 < n; r0 += SYM_H) {
      const int64_t H = std::min<int64_t>(SYM_H, n - r0);
      const int64_t e = panel_ext(n, r0, ext);
      const int64_t w = round_up(e, PADV);
      lb.poff.push_back((int64_t)elems);
      lb.pw.push_back(w);
      elems += (size_t)(H * w);
      valid += (double)H * (double)e;
    }
    lb.stored_bytes = valid * 8.0;
    HIPCHK(hipMalloc(&lb.d_poff, sizeof(int64_t) * lb.poff.size()));
    HIPCHK(hipMalloc(&lb.d_pw, sizeof(int64_t) * lb.pw.size()));
    HIPCHK(hipMemcpy(lb.d_poff, lb.poff.data(), sizeof(int64_t) * lb.poff.size(),
                     hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(lb.d_pw, lb.pw.data(), sizeof(int64_t) * lb.pw.size(), hipMemcpyHostToDevice));
  }
  {
    const hipError_t e = hipMalloc(&lb.ptr, sizeof(double) * elems);
    if (e != hipSuccess) {
      lb.ptr = nullptr;
      size_t fr = 0, tot = 0;
      (void)hipGetLastError();
      (void)hipMemGetInfo(&fr, &tot);
      return fail(c, SGV_ERR_HIP,
                  "LD matrix %d block %d (n=%lld, %s): %.2f GB of device memory needed, %.2f GB "
                  "free: %s", ld, b, (long long)n,
                  fmt == 0 ? "dense" : ext > 0 ? "packed band" : "packed triangle",
                  sizeof(double) * (double)elems / 1e9, (double)fr / 1e9, hipGetErrorString(e));
    }
  }
  HIPCHK(hipMemsetAsync(lb.ptr, 0, sizeof(double) * elems, c->st));
  BlkDesc d{fmt == 0 ? lb.ptr : nullptr, c->lda[b], c->bn[b], c->bvoff[b]};
  HIPCHK(hipMemcpyAsync(c->d_blks[ld] + b, &d, sizeof d, hipMemcpyHostToDevice, c->st));
  CHK(stream_wait(c));
  return SGV_OK;
}

static int ld_ready(sgv_ctx* c, int ld) {
  for (int b = 0; b < c->nblk; ++b)
    if (!c->ldb[ld][b].ptr)
      return fail(c, SGV_ERR_STATE, "LD matrix %d block %d has not been set", ld, b);
  return SGV_OK;
}

template <typename T>
static int upload_table(sgv_ctx* c, const std::vector<T>& h, T** d) {
  if (h.empty()) return SGV_OK;
  HIPCHK(hipMalloc(d, sizeof(T) * h.size()));
  HIPCHK(hipMemcpy(*d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  return SGV_OK;
}

static int grow(sgv_ctx* c, double** buf, size_t* cap, size_t need) {
  if (need <= *cap) return SGV_OK;
  if (*buf) HIPCHK(hipFree(*buf));
  *buf = nullptr;
  HIPCHK(hipMalloc(buf, sizeof(double) * need));
  *cap = need;
  return SGV_OK;
}


// panels per MFMA strip (env SGV_MFMA_STRIP, read when a plan is built; 1 =
// one (panel, chunk) item per workgroup)
static int mfma_strip_len() {
  const char* e = ab_env("SGV_MFMA_STRIP");
  const int v = e ? std::atoi(e) : 8;
  return std::max(1, std::min(64, v));
}

// Block groups of the MFMA pass (SGV_PASS_GROUPS with SGV_AB=1 forces a count):
// by default one group per ~4 rounds of strips on the device's workgroup slots,
// at most 4 -- a group's finalize then overlaps the next group's strips on a
// second stream.  The grouping changes no sum (strips and panels are the same
// work items in another launch), so products are bitwise the same for every
// count; it is a function of this rank's plan only.
static int pass_groups(int nstrips, int nblk, int slots) {
  const char* e = ab_env("SGV_PASS_GROUPS");
  int g = e ? std::atoi(e) : nstrips / std::max(1, 4 * slots);
  return std::max(1, std::min(std::min(g, 8), nblk));
}

static int device_cus() {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
      ncu = prop.multiProcessorCount;
  }
  return ncu;
}

// Longest-processing-time makespan of `cost` on `slots` identical slots, as a
// fraction of the perfect split (the dispatcher hands the strips out in this
// order, most panels first, to whichever slot frees first)
static double lpt_efficiency(std::vector<double> cost, int slots) {
  std::sort(cost.begin(), cost.end(), std::greater<double>());
  std::vector<double> load((size_t)slots, 0.0);
  double tot = 0.0;
  for (double x : cost) {
    auto it = std::min_element(load.begin(), load.end());
    *it += x;
    tot += x;
  }
  const double mk = *std::max_element(load.begin(), load.end());
  return mk > 0.0 ? tot / slots / mk : 1.0;
}

// NC <= 8 MFMA passes: the 4-wave kernel (two 4-wave workgroups per CU, 512
// slots) or the wave-pair kernel (one 8-wave workgroup per CU, a strip in half
// the time: 256 slots at half the cost) -- bitwise the same products, so the
// choice is free per plan.  Auto (1): the pair kernel for 3-4-column passes
// when its launch drains with at least 3 % less tail by the strips' model cost
// (a few strips per slot: an 8-block share of the north star); SGV_MF_PAIR=0 / 1
// (with SGV_AB=1) forces none / every 3-8-column pass (2).
static int mfma_pair_choice(const std::vector<SymStrip>& strips,
                            const std::vector<SymItem>& sitems) {
  const char* e = ab_env("SGV_MF_PAIR");
  if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1' ? 2 : 0;
  const int ncu = device_cus();
  std::vector<double> cost;
  cost.reserve(strips.size());
  for (const SymStrip& st : strips) {
    double x = 0.0;
    for (int i = 0; i < st.npan; ++i) x += (double)sitems[st.it0 + i].H / SYM_H;
    cost.push_back(x * (double)st.ncmax / 512.0);
  }
  const double quad = lpt_efficiency(cost, 2 * ncu);
  const double pair = lpt_efficiency(cost, ncu);   // per slot: twice the speed, same ratio
  return pair >= quad + 0.03 ? 1 : 0;
}

// MFMA strips of one LD matrix from the class-1 (512-column) tables.  Chunk
// (parity p, c0 = 256 p + 512 k) of a block holds the items (g, c0) of panels
// g = p, p + 2, ..., G = c0 / 256 (the diagonal panel); they are cut into strips
// of up to S panels in increasing order, colpart slots numbered per chunk.
// The chunk's strips hold the column sums of panel G's rows (offset 0, "own")
// and of panel G + 1's rows (offset 256, "other").  Dispatch order: by block
// group (pass_groups), then most panels first (the short strips fill the tail).
static int build_strips(sgv_ctx* c, int ld, const std::vector<SymItem>& items,
                        const std::vector<SymPanel>& panels, LdPlan* pl) {
  constexpr int cw = 512;
  const int S = mfma_strip_len();
  constexpr int NPAR = cw / SYM_H;   // 512-column chunks start at 256 p + 512 k
  std::vector<SymItem> sitems;
  std::vector<SymStrip> strips;
  std::vector<int> sblk;             // block of each strip (creation order)
  std::vector<SymPanel> sp = panels;
  std::vector<int> pblk(panels.size(), 0);
  int bp0 = 0;
  for (int b = 0; b < c->nblk; ++b) {
    if (c->ldb[ld][b].fmt != 1) continue;
    const int64_t n = c->bn[b];
    const int np = (int)c->ldb[ld][b].poff.size();
    for (int g = 0; g < np; ++g) pblk[bp0 + g] = b;
    for (int p = 0; p < NPAR; ++p)
      for (int64_t c0 = (int64_t)SYM_H * p; c0 < n; c0 += cw) {
        const int G = (int)(c0 / SYM_H);
        const int sb = (int)strips.size();
        // a band block's panel g reaches c0 iff c0 - 256 g < ext (ext = e
        // panels: the panels G - NPAR floor((e - 1) / NPAR), ..., G of this class)
        const int64_t ext = c->ldb[ld][b].ext;
        const int glo = ext > 0 ? std::max(p, G - NPAR * (((int)(ext / SYM_H) - 1) / NPAR)) : p;
        for (int g0 = glo; g0 <= G; g0 += NPAR * S) {
          SymStrip st;
          st.it0 = (int)sitems.size();
          st.npan = 0;
          st.slot = (int)strips.size();
          st.ncmax = 0;
          for (int g = g0; g <= G && g < g0 + NPAR * S; g += NPAR) {
            const SymPanel& pn = panels[bp0 + g];
            const int idx = pn.item_begin + (int)((c0 - (int64_t)SYM_H * g) / cw);
            if (idx >= pn.item_end || items[idx].c0 != c0)
              return fail(c, SGV_ERR_STATE, "strip plan: item (%d, %lld) missing", g,
                          (long long)c0);
            sitems.push_back(items[idx]);
            st.ncmax = std::max(st.ncmax, items[idx].nc);
            ++st.npan;
          }
          strips.push_back(st);
          sblk.push_back(b);
        }
        sp[bp0 + G].own_sb = sb;
        sp[bp0 + G].own_se = (int)strips.size();
        if (NPAR == 2 && G + 1 < np) {
          sp[bp0 + G + 1].oth_sb = sb;
          sp[bp0 + G + 1].oth_se = (int)strips.size();
        }
      }
    bp0 += np;
  }
  // block groups: contiguous blocks, balanced by stored bytes
  const int ncu = device_cus();
  std::vector<int> grp(c->nblk, 0);
  int ngrp = pass_groups((int)strips.size(), c->nblk, 2 * ncu);
  {
    double tot = 0.0;
    for (int b = 0; b < c->nblk; ++b) tot += c->ldb[ld][b].stored_bytes;
    double acc = 0.0;
    for (int b = 0; b < c->nblk; ++b) {
      grp[b] = std::min(ngrp - 1, (int)(acc / tot * ngrp));
      acc += c->ldb[ld][b].stored_bytes;
    }
    ngrp = grp[c->nblk - 1] + 1;
  }
  // group, then most panels first, creation order within a count.  Measured
  // slower (profiles/r03/s4/): ordering by stored bytes (2-10 %) and
  // XCD-contiguous eighths of the creation order (north star +5 %, 8 x 25,000
  // +4-7 %, the 8-block share -1 %)
  {
    std::vector<int> ord(strips.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int)i;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) {
      if (grp[sblk[x]] != grp[sblk[y]]) return grp[sblk[x]] < grp[sblk[y]];
      return strips[x].npan > strips[y].npan;
    });
    std::vector<SymStrip> o(strips.size());
    pl->gs.assign(ngrp + 1, 0);
    for (size_t i = 0; i < ord.size(); ++i) {
      o[i] = strips[ord[i]];
      pl->gs[grp[sblk[ord[i]]] + 1] = (int)i + 1;
    }
    for (int g = 1; g <= ngrp; ++g) pl->gs[g] = std::max(pl->gs[g], pl->gs[g - 1]);
    strips.swap(o);
  }
  // finalize dispatch order (a panel's sums do not depend on it): by group, then
  // most row and column parts first, so the one-item panels at the blocks' ends
  // fill the tail (NC = 16 -0.8 % per pass, profiles/r03/fin_lpt_ab.jsonl)
  {
    std::vector<int> ord(sp.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int)i;
    auto work = [&](const SymPanel& a) {
      return (a.item_end - a.item_begin) + (a.own_se - a.own_sb) + (a.oth_se - a.oth_sb);
    };
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) {
      if (grp[pblk[x]] != grp[pblk[y]]) return grp[pblk[x]] < grp[pblk[y]];
      return work(sp[x]) > work(sp[y]);
    });
    std::vector<SymPanel> o(sp.size());
    pl->gp.assign(ngrp + 1, 0);
    for (size_t i = 0; i < ord.size(); ++i) {
      o[i] = sp[ord[i]];
      pl->gp[grp[pblk[ord[i]]] + 1] = (int)i + 1;
    }
    for (int g = 1; g <= ngrp; ++g) pl->gp[g] = std::max(pl->gp[g], pl->gp[g - 1]);
    sp.swap(o);
  }
  pl->ngrp = ngrp;
  pl->nstrips = (int)strips.size();
  pl->ragged = false;
  for (const SymStrip& st : strips)
    for (int i = 0; i < st.npan; ++i) pl->ragged |= sitems[st.it0 + i].nc < st.ncmax;
  pl->pair = pl->ragged ? 0 : mfma_pair_choice(strips, sitems);
  CHK(upload_table(c, strips, &pl->d_strips));
  CHK(upload_table(c, sitems, &pl->d_sitems));
  CHK(upload_table(c, sp, &pl->d_spanels));
  return SGV_OK;
}

// rank holding global block gb (rank_blk0 from the communicator; -1 outside)
static int rank_of_block(const sgv_ctx* c, int gb) {
  const int nr = (int)c->rank_blk0.size() - 1;
  for (int r = 0; r < nr; ++r)
    if (gb >= c->rank_blk0[r] && gb < c->rank_blk0[r + 1]) return r;
  return -1;
}

// Coupling tasks of LD matrix ld and the panel slots they fill: for each
// coupling (gb, gb + 1) side 0 = gb's last nr rows (if gb is local), side 1 =
// gb + 1's first nc rows (if local), cut at panel boundaries; slot[(b, g)]
// numbers the panels holding such rows.  Sources on another rank come from the
// halo exchange (neighbouring ranks only: pieces are contiguous).
static int plan_couplings(sgv_ctx* c, int ld, LdPlan& pl, std::vector<int>& slot_of,
                          std::vector<int>& slot_base) {
  const std::vector<LdCoupling>& cv = c->cpl[ld];
  slot_base.assign(c->nblk + 1, 0);
  for (int b = 0; b < c->nblk; ++b)
    slot_base[b + 1] = slot_base[b] + (int)std::max<size_t>(1, c->ldb[ld][b].poff.size());
  slot_of.assign(slot_base[c->nblk], -1);
  if (cv.empty()) return SGV_OK;
  const int me = c->rank;
  std::vector<CouplingTask> tasks;
  int ncp = 0;
  auto slot = [&](int b, int g) {
    int& sref = slot_of[slot_base[b] + g];
    if (sref < 0) sref = ncp++;
    return sref;
  };
  pl.hmax = 0;
  for (const LdCoupling& q : cv) pl.hmax = std::max<int64_t>(pl.hmax, std::max(q.nr, q.nc));
  pl.halo = false;
  pl.h_len0 = pl.h_len1 = 0;
  for (const LdCoupling& q : cv) {
    const int ra = rank_of_block(c, q.gb), rb = rank_of_block(c, q.gb + 1);
    if (ra < 0 || rb < 0)
      return fail(c, SGV_ERR_STATE, "coupling (%d, %d): block outside the partition", q.gb, q.gb + 1);
    if (ra != rb) pl.halo = true;   // the same decision on every rank
    const int ba = q.gb - c->blk0, bb = q.gb + 1 - c->blk0;
    const bool la = ba >= 0 && ba < c->nblk, lb = bb >= 0 && bb < c->nblk;
    if (ra != rb && la) {           // gb is this rank's last block: send its tail
      pl.h_src1 = c->bvoff[ba] + c->bn[ba] - q.nr;
      pl.h_len1 = q.nr;
    }
    if (ra != rb && lb) {           // gb + 1 is this rank's first block: send its head
      pl.h_src0 = c->bvoff[bb];
      pl.h_len0 = q.nc;
    }
    if (la && c->ldb[ld][ba].fmt != 1)
      return fail(c, SGV_ERR_ARG, "coupling (%d, %d): pieces must be stored packed", q.gb, q.gb + 1);
    if (lb && c->ldb[ld][bb].fmt != 1)
      return fail(c, SGV_ERR_ARG, "coupling (%d, %d): pieces must be stored packed", q.gb, q.gb + 1);
    for (int side = 0; side < 2; ++side) {
      if (side == 0 && !la) continue;
      if (side == 1 && !lb) continue;
      const int b = side == 0 ? ba : bb;
      const int64_t rbeg = side == 0 ? c->bn[b] - q.nr : 0;   // block-relative output rows
      const int64_t rend = side == 0 ? c->bn[b] : q.nc;
      for (int64_t r = rbeg; r < rend;) {
        const int g = (int)(r / SYM_H);
        const int64_t pe = std::min<int64_t>(rend, (int64_t)(g + 1) * SYM_H);
        CouplingTask t;
        t.m = side == 0 ? q.d_up : q.d_lo;
        t.ldm = side == 0 ? q.nr : q.nc;
        t.inner = side == 0 ? q.nc : q.nr;
        t.row0 = (int32_t)(r - rbeg);
        t.nrows = (int32_t)(pe - r);
        t.cp = slot(b, g);
        t.prow0 = (int32_t)(r - (int64_t)g * SYM_H);
        const bool local_src = side == 0 ? lb : la;
        t.local = local_src ? 1 : 0;
        if (local_src)
          t.src = side == 0 ? c->bvoff[bb] : c->bvoff[ba] + c->bn[ba] - q.nr;
        else   // halo [rank][slot]: the next rank's head (slot 0) or the previous one's tail (1)
          t.src = side == 0 ? 2 * (int64_t)rb + 0 : 2 * (int64_t)ra + 1;
        tasks.push_back(t);
        r = pe;
      }
      pl.cpl_bytes += 8.0 * q.nr * q.nc;
    }
  }
  (void)me;
  pl.nctasks = (int)tasks.size();
  pl.ncp = ncp;
  CHK(upload_table(c, tasks, &pl.d_ctasks));
  CHK(grow(c, &c->d_cpbuf, &c->cpbuf_cap, (size_t)std::max(ncp, 1) * 256 * MAXC));
  if (pl.halo) {
    const size_t per = 2 * (size_t)MAXC * pl.hmax;
    CHK(grow(c, &c->d_halo, &c->halo_cap, per * (1 + (size_t)c->nranks)));
    if (c->host_ag && c->h_halo_cap < per * (1 + (size_t)c->nranks)) {
      if (c->h_halo) HIPCHK(hipHostFree(c->h_halo));
      c->h_halo = nullptr;
      HIPCHK(hipHostMalloc(&c->h_halo, sizeof(double) * per * (1 + (size_t)c->nranks)));
      c->h_halo_cap = per * (1 + (size_t)c->nranks);
    }
    if (!c->comm && !c->host_ag)
      return fail(c, SGV_ERR_STATE, "a coupling spans two ranks but no communicator is set");
  }
  return SGV_OK;
}

// launch tables of LD matrix ld: dense row groups, packed (panel, chunk) items
// per chunk-width class, panels; unified partial slots in block order
static int ensure_plan(sgv_ctx* c, int ld) {
  LdPlan& pl = c->plan[ld];
  if (pl.valid) return SGV_OK;
  CHK(ld_ready(c, ld));
  free_plan(pl);
  std::vector<RowGroup> rg;
  std::vector<int> pbeg(c->nblk + 1, 0);
  const int rows = ld_pass_rows_per_group();
  int nparts = 0;
  for (int b = 0; b < c->nblk; ++b) {
    const LdBlock& lb = c->ldb[ld][b];
    pbeg[b] = nparts;
    pl.stored_bytes += lb.stored_bytes;
    pl.dense_bytes += (double)c->bn[b] * (double)c->bn[b] * 8.0;
    if (lb.fmt == 0) {
      for (int64_t r0 = 0; r0 < c->bn[b]; r0 += rows) rg.push_back(RowGroup{b, (int32_t)r0, nparts++, 0});
    } else {
      nparts += (int)lb.poff.size();   // one slot per panel
    }
  }
  pbeg[c->nblk] = nparts;
  pl.nparts = nparts;
  pl.nrg = (int)rg.size();
  CHK(upload_table(c, rg, &pl.d_rg));
  CHK(upload_table(c, pbeg, &pl.d_pbeg));
  std::vector<int> cp_slot, cp_base;   // coupled band pieces: panel -> cpbuf slot
  CHK(plan_couplings(c, ld, pl, cp_slot, cp_base));
  size_t rowpart_need = 0, colpart_need = 0;
  for (int cls = 0; cls < 4; ++cls) {
    const int cw = 1024 >> cls;
    std::vector<SymItem> items;
    std::vector<SymPanel> panels;
    for (int b = 0; b < c->nblk; ++b) {
      const LdBlock& lb = c->ldb[ld][b];
      if (lb.fmt != 1) continue;
      const int64_t n = c->bn[b];
      const int blk_panel0 = (int)panels.size();
      for (size_t g = 0; g < lb.poff.size(); ++g) {
        const int r0 = (int)(g * SYM_H);
        const int H = (int)std::min<int64_t>(SYM_H, n - r0);
        const int ib = (int)items.size();
        const int64_t cend = r0 + panel_ext(n, r0, lb.ext);
        for (int64_t c0 = r0; c0 < cend; c0 += cw) {
          SymItem it;
          it.P = lb.ptr + lb.poff[g];
          it.w = lb.pw[g];
          it.voff = c->bvoff[b];
          it.r0 = r0;
          it.H = H;
          it.c0 = (int32_t)c0;
          it.nc = (int32_t)std::min<int64_t>(cw, cend - c0);
          it.item = (int32_t)items.size();
          it.diag_end = r0 + H;
          items.push_back(it);
        }
        SymPanel pn;
        pn.voff = c->bvoff[b];
        pn.r0 = r0;
        pn.H = H;
        pn.item_begin = ib;
        pn.item_end = (int)items.size();
        pn.g = (int)g;
        pn.blk_panel0 = blk_panel0;
        pn.part = pbeg[b] + (int)g;
        // first earlier panel whose stored columns cover this panel's rows
        pn.gmin = lb.ext > 0 ? std::max<int>(0, (int)g - (int)(lb.ext / SYM_H) + 1) : 0;
        pn.own_sb = pn.own_se = pn.oth_sb = pn.oth_se = 0;
        pn.cp = cp_slot[cp_base[b] + (int)g];
        panels.push_back(pn);
      }
    }
    pl.nitems[cls] = (int)items.size();
    pl.npanels = (int)panels.size();
    {
      // dispatch order: largest items first (rows x columns), so the small edge
      // items fill the tail of the launch; the `item` field keeps the partial slot
      std::vector<SymItem> order = items;
      std::stable_sort(order.begin(), order.end(), [](const SymItem& a, const SymItem& b) {
        return (int64_t)a.H * a.nc > (int64_t)b.H * b.nc;
      });
      CHK(upload_table(c, order, &pl.d_items[cls]));
    }
    CHK(upload_table(c, panels, &pl.d_panels[cls]));
    if (cls == 1) CHK(build_strips(c, ld, items, panels, &pl));
    const size_t ncmax = (size_t)sym_class_nc(cls);
    rowpart_need = std::max(rowpart_need, items.size() * SYM_H * ncmax);
    colpart_need = std::max(colpart_need, items.size() * ncmax * (size_t)cw);
  }
  if (pl.npanels) {   // the MFMA pass: class-1 items with up to 16 columns
    rowpart_need = std::max(rowpart_need, (size_t)pl.nitems[1] * SYM_H * MAXC);
    colpart_need = std::max(colpart_need, (size_t)pl.nstrips * MAXC * 512);
    CHK(grow(c, &c->d_pk, &c->pk_cap, (size_t)c->Mpad * 16));
  }
  CHK(grow(c, &c->d_rowpart, &c->rowpart_cap, rowpart_need));
  CHK(grow(c, &c->d_colpart, &c->colpart_cap, colpart_need));
  CHK(grow(c, &c->d_part, &c->part_cap, (size_t)nparts * MAXC));
  pl.valid = true;
  return SGV_OK;
}

static const int* ld_parts(sgv_ctx* c, int ld) { return c->plan[ld].d_pbeg; }

static int gather_f64(sgv_ctx* c, const double* d_send, double* d_recv, size_t cnt,
                      double* h_send, double* h_recv);

// coupling sums of LD matrix ld's band pieces for this pass (before the
// finalize that adds them): the halo of a coupling that spans two ranks is
// all-gathered first (every rank takes part, whatever its own couplings)
static int coupling_pass(sgv_ctx* c, const LdPlan& pl, int nc, const PassArgs& pa) {
  const double* recv = nullptr;
  if (pl.halo) {
    const size_t per = 2 * (size_t)nc * pl.hmax;
    double* send = c->d_halo;
    double* drecv = c->d_halo + per;
    HIPCHK(launch_halo_pack(pa, nc, pl.h_src0, pl.h_len0, pl.h_src1, pl.h_len1, pl.hmax, send,
                            c->st));
    CHK(gather_f64(c, send, drecv, per, c->h_halo, c->h_halo ? c->h_halo + per : nullptr));
    recv = drecv;
  }
  if (pl.nctasks)
    HIPCHK(launch_coupling(nc, pl.d_ctasks, pl.nctasks, pa, recv, pl.hmax, c->d_cpbuf, pl.ncp,
                           c->st));
  c->aux_bytes += pl.cpl_bytes + 2.0 * 8.0 * nc * 256.0 * pl.ncp;
  return SGV_OK;
}

static int ld_pass(sgv_ctx* c, int ld, int nc, const PassArgs& pa_in) {
  if (nc <= 0) return SGV_OK;
  CHK(ensure_plan(c, ld));
  const LdPlan& pl = c->plan[ld];
  PassArgs pa = pa_in;
  pa.cpbuf = c->d_cpbuf;
  hipEvent_t e0, e1;
  if (c->evpool.size() < 2) {
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
  } else {
    e0 = c->evpool.back();
    c->evpool.pop_back();
    e1 = c->evpool.back();
    c->evpool.pop_back();
  }
  HIPCHK(hipEventRecord(e0, c->st));
  if (pl.halo || pl.nctasks) CHK(coupling_pass(c, pl, nc, pa));
  if (pl.nrg) HIPCHK(launch_ld_pass(nc, c->d_blks[ld], pl.d_rg, pl.nrg, pa, c->d_part, c->st));
  if (pl.npanels) {
    const bool mf = c->mfma_min > 0 && nc >= c->mfma_min;
    const int cls = mf ? 1 : sym_class(nc);
    if (mf) {
      HIPCHK(launch_pk(pa, nc, c->Mpad, c->d_pk, c->st));
      if (pl.ngrp <= 1) {
        HIPCHK(launch_sym_mfma(nc, pl.d_strips, pl.nstrips, pl.d_sitems, pa, c->d_pk,
                               c->d_rowpart, c->d_colpart, pl.ragged, pl.pair, c->st));
        HIPCHK(launch_sym_finalize_strip(nc, pl.d_spanels, pl.npanels, pa, c->d_rowpart,
                                         c->d_colpart, c->d_part, pl.ragged, c->st));
      } else {
        // group g's strips on the ctx stream, its finalize on the side stream
        // behind them: the finalize (and the launch tail) of g overlaps g + 1's
        // strips.  Same work items, so the products are bitwise the one-launch
        // pass's; the pass's events (e0 on st, e1 after the join) span both
        for (int g = 0; g < pl.ngrp; ++g) {
          HIPCHK(launch_sym_mfma(nc, pl.d_strips + pl.gs[g], pl.gs[g + 1] - pl.gs[g],
                                 pl.d_sitems, pa, c->d_pk, c->d_rowpart, c->d_colpart, pl.ragged,
                                 pl.pair, c->st));
          HIPCHK(hipEventRecord(c->ev_grp[g % MAXGRP], c->st));
          HIPCHK(hipStreamWaitEvent(c->st_fin, c->ev_grp[g % MAXGRP], 0));
          HIPCHK(launch_sym_finalize_strip(nc, pl.d_spanels + pl.gp[g], pl.gp[g + 1] - pl.gp[g],
                                           pa, c->d_rowpart, c->d_colpart, c->d_part, pl.ragged,
                                           c->st_fin));
        }
        HIPCHK(hipEventRecord(c->ev_fin, c->st_fin));
        HIPCHK(hipStreamWaitEvent(c->st, c->ev_fin, 0));
      }
      c->aux_bytes += 2.0 * 8.0 * nc * ((double)pl.nitems[cls] * SYM_H +
                                        (double)pl.nstrips * 512);
      c->aux_bytes += 8.0 * (double)c->Mpad * ((nc <= 4 ? 4 : nc <= 8 ? 8 : 16) + nc);   // Pk pack
    } else {
      HIPCHK(launch_sym_pass(nc, cls, pl.d_items[cls], pl.nitems[cls], pa, c->d_rowpart,
                             c->d_colpart, c->st));
      HIPCHK(launch_sym_finalize(nc, cls, pl.d_panels[cls], pl.npanels, pa, c->d_rowpart,
                                 c->d_colpart, c->d_part, c->st));
      const double cw = (double)(1024 >> cls);
      c->aux_bytes += 2.0 * 8.0 * nc * (double)pl.nitems[cls] * (SYM_H + cw);
    }
  }
  HIPCHK(hipEventRecord(e1, c->st));
  c->pending.emplace_back(e0, e1);
  c->ld_launches += 1.0;
  c->ld_bytes += pl.stored_bytes;
  c->dense_bytes += pl.dense_bytes;
  c->rhs_bytes += 2.0 * nc * (double)c->Mloc * 8.0;
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// batched CG (scipy 1.15.3, iterative.py:375-422) on columns 0..ncol-1.
// On entry: X = x0, Rr = P = r0 (= b - A x0 or b), rho[c] = r0.r0,
// atol[c] = rtol*|b|.  Columns with active[c] = 0 are skipped (bnrm2 == 0).
// Column c uses LD matrix col_ld[c] and A = c1[c] R + c2[c] I.
// ---------------------------------------------------------------------------
struct CgCols {
  int ncol = 0;
  int col_ld[MAXC];
  double c1[MAXC], c2[MAXC];
  double* X[MAXC];
  double* Rr[MAXC];
  double* P[MAXC];
  double* Q[MAXC];
  double* RX[MAXC] = {};   // non-null: carry R_s x (RX += alpha R_s p), Y = R_s p scratch
  double* Y[MAXC] = {};
  double s = 0.0;          // ridge of R_s
};

static int cg_loop(sgv_ctx* c, const CgCols& cc, double* rho, const double* atol, int maxiter,
                   const int* active_in, int* iters, int* info, int* passes) {
  const int ncol = cc.ncol;
  int active[MAXC];
  double rho_prev[MAXC];
  for (int j = 0; j < ncol; ++j) {
    active[j] = active_in[j];
    rho_prev[j] = 0.0;
    if (!active[j]) {
      iters[j] = 0;
      info[j] = 0;
    }
  }
  for (int it = 0; it < maxiter; ++it) {
    unsigned mask = 0;
    for (int j = 0; j < ncol; ++j) {
      if (!active[j]) continue;
      if (std::sqrt(rho[j]) < atol[j]) {  // iterative.py:398 (strict <)
        active[j] = 0;
        iters[j] = it;
        info[j] = 0;
        continue;
      }
      mask |= 1u << j;
    }
    if (!mask) return SGV_OK;
    if (it > 0) {  // iterative.py:403-407
      PArgs pa{};
      pa.ncol = ncol;
      pa.mask = mask;
      for (int j = 0; j < ncol; ++j) {
        pa.P[j] = cc.P[j];
        pa.Rr[j] = cc.Rr[j];
        pa.beta[j] = (mask >> j & 1u) ? rho[j] / rho_prev[j] : 0.0;
      }
      HIPCHK(launch_cg_p(c->d_ch, c->nch, pa, c->st));
    }
    // q = A p (iterative.py:411): one pass per LD matrix over its active columns
    for (int ld = 0; ld < c->nld; ++ld) {
      PassArgs pa{};
      Map16 map = identity_map();
      int nc = 0;
      for (int j = 0; j < ncol; ++j) {
        if (!(mask >> j & 1u) || cc.col_ld[j] != ld) continue;
        pa.in[nc] = cc.P[j];
        pa.out[nc] = cc.Q[j];
        pa.dot[nc] = cc.P[j];
        pa.yout[nc] = cc.RX[j] ? cc.Y[j] : nullptr;
        pa.c1[nc] = cc.c1[j];
        pa.c2[nc] = cc.c2[j];
        map.d[nc] = j;
        ++nc;
      }
      if (!nc) continue;
      pa.ys1 = 1.0 - cc.s;   // Y = R_s p = (1-s) R p + s p
      pa.ys0 = cc.s;
      CHK(ld_pass(c, ld, nc, pa));
      CHK(reduce_dev(c, nc, ld_parts(c, ld), map, c->d_pq));
      if (passes) ++*passes;
    }
    // alpha = rho / p.q; x += alpha p; r -= alpha q; rho_new = r.r (:412-415)
    XrArgs xa{};
    xa.ncol = ncol;
    xa.mask = mask;
    xa.pq = c->d_pq;
    for (int j = 0; j < ncol; ++j) {
      xa.X[j] = cc.X[j];
      xa.Rr[j] = cc.Rr[j];
      xa.P[j] = cc.P[j];
      xa.Q[j] = cc.Q[j];
      xa.RX[j] = cc.RX[j];
      xa.Y[j] = cc.Y[j];
      xa.rho[j] = rho[j];
    }
    HIPCHK(launch_cg_xr(c->d_ch, c->nch, xa, c->d_part, c->st));
    double rn[MAXC];
    CHK(reduce_host(c, MAXC, c->d_ch_begin, rn));
    for (int j = 0; j < ncol; ++j)
      if (mask >> j & 1u) {
        rho_prev[j] = rho[j];
        rho[j] = rn[j];
      }
  }
  for (int j = 0; j < ncol; ++j)
    if (active[j]) {  // for-loop exhausted (iterative.py:420-422)
      iters[j] = maxiter;
      info[j] = maxiter;
    }
  return SGV_OK;
}

// spin on an event already recorded on the ctx stream
static int event_spin(sgv_ctx* c, hipEvent_t ev) {
  hipError_t e;
  while ((e = hipEventQuery(ev)) == hipErrorNotReady) __builtin_ia32_pause();
  if (e != hipSuccess) return fail(c, SGV_ERR_HIP, "event wait: %s", hipGetErrorString(e));
  return SGV_OK;
}

// Pipelined CG: the iteration of cg_loop with the stop test, beta and alpha on
// the device, so no host round trip sits between two iterations.  Iteration it
// is enqueued as [k_cg_ctl (stop test of `it`, beta), p update, LD pass(es) +
// p.q, x/r update + r.r]; the p/x/r kernels and the passes read the device
// state and become no-ops once no column is active.  The host then waits only
// for k_cg_ctl of `it` (the first kernel of the iteration: the wait overlaps
// the pass) and enqueues it + 1 behind it with the columns still active after
// that test -- so the column set of every pass is a function of the trajectory
// alone (deterministic; a column stopping at it + 1's test rides along in that
// pass unused).  When the test of `it` stops every column, that iteration's
// kernels were no-ops: their pass timers and byte counts are dropped.
// Exact column sets (default, from it = 1): the p update of `it` (a no-op for
// the columns the device state has stopped) is enqueued first, then the host
// waits for the test of `it` -- it completes while that p update runs -- and
// enqueues the passes with the columns still active after it.  A CG #1 column
// that stops one iteration before its CG #2 partner then leaves the pass
// (north star: NC 8 -> 4, one pass in three once the iteration counts split;
// the same iterates bit for bit there).  Where the smaller set crosses a kernel
// boundary (NC <= 2 runs the VALU pass, 3..16 the MFMA pass) the surviving
// columns' sums are formed in another order: equal to rounding.
// With a communicator the CG prologue's sums (|b|^2, |r0|^2: the LMMSE init
// kernel's partials, `m0`) ride in the exchange of iteration 0's p.q instead of
// one of their own: the first pass runs on p0 = r0 for every column before the
// stop test of iteration 0 is known (as the look-ahead pass does), then
// k_cg_init and the test follow the shared reduction.  Same values, one
// exchange fewer per LMMSE; only where one LD matrix serves every column.
struct CgMerge0 {
  const double* part = nullptr;   // [chunk][2 MAXC] (k_lmmse_init)
  double rtol = 0.0;
  double* const* X = nullptr;     // k_cg_init zeroes X, R_s X of |b| == 0 columns
  double* const* RX = nullptr;
};

static int cg_loop_dev(sgv_ctx* c, const CgCols& cc, const double* rho0, const double* atol,
                       int maxiter, const int* active_in, int* iters, int* info, int* passes,
                       const CgMerge0* m0 = nullptr) {
  const int ncol = cc.ncol;
  unsigned mask = 0;
  if (rho0) {
    CgState* hi = c->h_cgi;   // the previous solve's copy has completed (its mirror was read)
    std::memset(hi, 0, sizeof(CgState));
    for (int j = 0; j < ncol; ++j) {
      hi->rho[j] = rho0[j];
      hi->atol[j] = atol[j];
      hi->active[j] = active_in[j] ? 1 : 0;
      if (active_in[j]) mask |= 1u << j;
    }
    hi->any = mask ? 1 : 0;
    HIPCHK(hipMemcpyAsync(c->d_cgs, hi, sizeof(CgState), hipMemcpyHostToDevice, c->st));
  } else {
    // state set by k_cg_init on the stream; a |b| == 0 column is inactive there
    // and rides along unused in the first pass (its result is never read)
    mask = ncol >= 32 ? ~0u : (1u << ncol) - 1u;
  }
  const volatile CgState* last = nullptr;
  int executed = 0;
  // one rank: iteration it's r.r reduction and the control of it + 1 are one
  // launch (k_cg_reduce_ctl), enqueued at the end of it, when that one
  // workgroup's reduction is short (fused_ctl_pays); SGV_EM_FUSE=0 A/B
  const bool fuse = !c->comm && !c->host_ag && fused_ctl_pays(MAXC, c->nblk);
  // exact sets pay only where fewer columns make a pass cheaper: the MFMA pass
  // (>= 3 columns of one LD matrix, cost by groups of 4); the VALU pass costs
  // the same at 1 and 2 columns (C2: 3.19 vs 3.21 ms), so K = 1 and distinct-LD
  // pairs keep the look-ahead and its host read stays off the critical path
  int widest = 0;
  double wide_bytes = 0.0;   // largest pass of >= 3 columns (this rank's blocks)
  for (int j = 0; j < ncol; ++j) {
    int n = 0;
    for (int i = 0; i < ncol; ++i) n += cc.col_ld[i] == cc.col_ld[j];
    widest = std::max(widest, n);
    if (n >= 3 && c->cg_exact < 0 && !c->comm && !c->host_ag) {
      CHK(ensure_plan(c, cc.col_ld[j]));
      wide_bytes = std::max(wide_bytes, c->plan[cc.col_ld[j]].stored_bytes);
    }
  }
  const bool exact = widest >= 3 && (c->cg_exact > 0 || (c->cg_exact < 0 && !c->comm &&
                                                         !c->host_ag &&
                                                         wide_bytes >= CG_EXACT_MIN_BYTES));
  for (int it = 0; it < maxiter; ++it) {
    const size_t np0 = c->pending.size();
    const double cnt0[5] = {c->ld_launches, c->ld_bytes, c->dense_bytes, c->rhs_bytes,
                            c->aux_bytes};
    int npass = 0;
    CgState* slot = c->h_cgm + (it % CG_RING);
    const bool merge = m0 && it == 0;   // the prologue's sums ride with this p.q
    if ((it == 0 || !fuse) && !merge) {
      HIPCHK(launch_cg_ctl(c->d_cgs, slot, c->d_rhonew, it, ncol, -1, c->st));
      HIPCHK(hipEventRecord(c->ev_cg[it % CG_RING], c->st));
    }
    if (it > 0) {  // iterative.py:403-407
      PArgs pa{};
      pa.ncol = ncol;
      pa.mask = mask;
      pa.st = c->d_cgs;
      for (int j = 0; j < ncol; ++j) {
        pa.P[j] = cc.P[j];
        pa.Rr[j] = cc.Rr[j];
      }
      HIPCHK(launch_cg_p(c->d_ch, c->nch, pa, c->st));
    }
    const bool pre = exact && it > 0;   // the test of `it` read before its passes
    if (pre) {
      const auto tw = std::chrono::steady_clock::now();
      CHK(event_spin(c, c->ev_cg[it % CG_RING]));
      c->host_wait_ms +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
      last = slot;
      if (!last->any) break;            // only the (no-op) p update was enqueued
      mask = 0;
      for (int j = 0; j < ncol; ++j)
        if (last->active[j]) mask |= 1u << j;
    }
    // q = A p (iterative.py:411): one pass per LD matrix over its columns
    for (int ld = 0; ld < c->nld; ++ld) {
      PassArgs pa{};
      Map16 map = identity_map();
      int nc = 0;
      for (int j = 0; j < ncol; ++j) {
        if (!(mask >> j & 1u) || cc.col_ld[j] != ld) continue;
        pa.in[nc] = cc.P[j];
        pa.out[nc] = cc.Q[j];
        pa.dot[nc] = cc.P[j];
        pa.yout[nc] = cc.RX[j] ? cc.Y[j] : nullptr;
        pa.c1[nc] = cc.c1[j];
        pa.c2[nc] = cc.c2[j];
        map.d[nc] = j;
        ++nc;
      }
      if (!nc) continue;
      pa.ys1 = 1.0 - cc.s;   // Y = R_s p = (1-s) R p + s p
      pa.ys0 = cc.s;
      pa.run = merge ? nullptr : &c->d_cgs->any;   // merge: the state is set after it
      CHK(ld_pass(c, ld, nc, pa));
      if (merge) {   // [|b|^2, |r0|^2] -> d_tot[0 .. 2 MAXC), p.q -> d_tot[2 MAXC + j]
        CHK(reduce_dev2(c, m0->part, 2 * MAXC, c->d_ch_begin, nc, ld_parts(c, ld), map, 2 * MAXC,
                        c->d_tot));
        HIPCHK(launch_cg_init(c->d_cgs, c->d_tot, m0->rtol, ncol, c->d_ch, c->nch, m0->X, m0->RX,
                              c->st));
        HIPCHK(launch_cg_ctl(c->d_cgs, slot, c->d_rhonew, it, ncol, -1, c->st));
        HIPCHK(hipEventRecord(c->ev_cg[it % CG_RING], c->st));
      } else {
        CHK(reduce_dev(c, nc, ld_parts(c, ld), map, c->d_pq));
      }
      ++npass;
    }
    // alpha = rho / p.q; x += alpha p; r -= alpha q; r.r (:412-415)
    XrArgs xa{};
    xa.ncol = ncol;
    xa.mask = mask;
    xa.pq = merge ? c->d_tot + 2 * MAXC : c->d_pq;
    xa.st = c->d_cgs;
    for (int j = 0; j < ncol; ++j) {
      xa.X[j] = cc.X[j];
      xa.Rr[j] = cc.Rr[j];
      xa.P[j] = cc.P[j];
      xa.Q[j] = cc.Q[j];
      xa.RX[j] = cc.RX[j];
      xa.Y[j] = cc.Y[j];
    }
    HIPCHK(launch_cg_xr(c->d_ch, c->nch, xa, c->d_part, c->st));
    if (fuse && it + 1 < maxiter) {
      HIPCHK(launch_cg_reduce_ctl(c->d_part, c->d_ch_begin, c->nblk, c->d_cgs,
                                  c->h_cgm + ((it + 1) % CG_RING), it + 1, ncol, c->st));
      HIPCHK(hipEventRecord(c->ev_cg[(it + 1) % CG_RING], c->st));
    } else {
      CHK(reduce_dev(c, MAXC, c->d_ch_begin, identity_map(), c->d_rhonew));
    }
    if (pre) {
      ++executed;
      if (passes) *passes += npass;
      continue;
    }
    // the stop test of `it` (its first kernel) decides whether it did any work
    CHK(event_spin(c, c->ev_cg[it % CG_RING]));
    last = slot;
    if (!last->any) {
      while (c->pending.size() > np0) {   // no-op passes: not timed, not counted
        c->evpool.push_back(c->pending.back().first);
        c->evpool.push_back(c->pending.back().second);
        c->pending.pop_back();
      }
      c->ld_launches = cnt0[0];
      c->ld_bytes = cnt0[1];
      c->dense_bytes = cnt0[2];
      c->rhs_bytes = cnt0[3];
      c->aux_bytes = cnt0[4];
      break;
    }
    ++executed;
    if (passes) *passes += npass;
    mask = 0;
    for (int j = 0; j < ncol; ++j)
      if (last->active[j]) mask |= 1u << j;
  }
  if (executed == maxiter) {  // for-loop exhausted (iterative.py:420-422)
    CgState* slot = c->h_cgm + (maxiter % CG_RING);
    HIPCHK(launch_cg_ctl(c->d_cgs, slot, c->d_rhonew, maxiter, ncol, maxiter, c->st));
    HIPCHK(hipEventRecord(c->ev_cg[maxiter % CG_RING], c->st));
    CHK(event_spin(c, c->ev_cg[maxiter % CG_RING]));
    last = slot;
  }
  for (int j = 0; j < ncol; ++j) {
    iters[j] = last->iters[j];
    info[j] = last->info[j];
  }
  return SGV_OK;
}

static int cg_run(sgv_ctx* c, const CgCols& cc, double* rho, const double* atol, int maxiter,
                  const int* active, int* iters, int* info, int* passes) {
  if (c->cg_pipe) return cg_loop_dev(c, cc, rho, atol, maxiter, active, iters, info, passes);
  return cg_loop(c, cc, rho, atol, maxiter, active, iters, info, passes);
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
  for (auto& pr : c->pending) {
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
static int gather_f64(sgv_ctx* c, const double* d_send, double* d_recv, size_t cnt,
                      double* h_send, double* h_recv) {
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
// SGV_XCHG_LAT_US (rank 0's value), or measured (sgv_exchange_probe).
// SGV_EM_REP=0/1 (with SGV_AB=1) forces either mode.
constexpr double EM_K_FIX_US = 5.0, EM_K_PER_CM_US = 1.1e-5, EM_T_REP_US = 35.0,
                 EM_T_PS_US = 15.0, EM_AG_GBS = 100.0;
static void em_costs(const sgv_ctx* c, double steps, double* rep_us, double* ps_us) {
  const double km = (double)c->K * (double)c->Mtot, n = (double)c->nranks, L = c->xlat_us;
  *rep_us = L + 8.0 * km * (n - 1.0) / n / (EM_AG_GBS * 1e3) +
            steps * (EM_K_FIX_US + EM_K_PER_CM_US * km + EM_T_REP_US);
  *ps_us = steps * (EM_K_FIX_US + EM_K_PER_CM_US * km / n + EM_T_PS_US + L);
}
// the mode of the next EM loop (maxit steps at most); records the prediction
static bool em_mode_pick(sgv_ctx* c, int maxit) {
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
static int gather_r1(sgv_ctx* c) {
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

// ---------------------------------------------------------------------------
// inputs
// ---------------------------------------------------------------------------
// exact symmetry test (tiled for cache locality)
static bool host_symmetric(const double* A, int64_t n, int64_t ld) {
  const int64_t T = 64;
  for (int64_t i0 = 0; i0 < n; i0 += T)
    for (int64_t j0 = i0; j0 < n; j0 += T)
      for (int64_t i = i0; i < std::min(n, i0 + T); ++i)
        for (int64_t j = std::max(j0, i + 1); j < std::min(n, j0 + T); ++j)
          if (!(A[i * ld + j] == A[j * ld + i])) return false;
  return true;
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

extern "C" int sgv_set_ld_packing(sgv_ctx* c, int mode) {
  ENTER(c);
  if (mode != 0 && mode != 1) return fail(c, SGV_ERR_ARG, "packing mode %d", mode);
  c->packing = mode;
  return SGV_OK;
}

extern "C" int sgv_set_ld_block(sgv_ctx* c, int ld, int b, const double* host, int64_t ld_host) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || b < 0 || b >= c->nblk || !host || ld_host < c->bn[b])
    return fail(c, SGV_ERR_ARG, "sgv_set_ld_block: bad arguments (ld=%d b=%d)", ld, b);
  const int64_t n = c->bn[b];
  const int fmt = (c->packing && host_symmetric(host, n, ld_host)) ? 1 : 0;
  CHK(ld_alloc(c, ld, b, fmt));
  const LdBlock& lb = c->ldb[ld][b];
  if (fmt == 0) {
    HIPCHK(hipMemcpy2D(lb.ptr, sizeof(double) * c->lda[b], host, sizeof(double) * ld_host,
                       sizeof(double) * n, n, hipMemcpyHostToDevice));
  } else {
    for (size_t g = 0; g < lb.poff.size(); ++g) {
      const int64_t r0 = (int64_t)g * SYM_H, H = std::min<int64_t>(SYM_H, n - r0);
      HIPCHK(hipMemcpy2D(lb.ptr + lb.poff[g], sizeof(double) * lb.pw[g], host + r0 * ld_host + r0,
                         sizeof(double) * ld_host, sizeof(double) * (n - r0), H,
                         hipMemcpyHostToDevice));
    }
  }
  std::fill(c->rx0_valid.begin(), c->rx0_valid.end(), 0);
  return SGV_OK;
}

// Upper triangle (diagonal included) of a symmetric LD block as CSR, block-
// relative: row i holds columns indices[indptr[i] .. indptr[i+1]) (each >= i,
// duplicates summed).  Stored packed; when the entries stay within a band
// j - i <= bw and the band's panels are narrower than the triangle, only the
// band is stored (panel extent round_up(256 + bw, BAND_Q) columns).  Panels
// are assembled in pinned host memory one at a time, no n x n buffer.
extern "C" int sgv_set_ld_block_csr(sgv_ctx* c, int ld, int b, const int64_t* indptr,
                                    const int64_t* indices, const double* data) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || b < 0 || b >= c->nblk || !indptr)
    return fail(c, SGV_ERR_ARG, "sgv_set_ld_block_csr: bad arguments (ld=%d b=%d)", ld, b);
  const int64_t n = c->bn[b];
  if (indptr[n] > 0 && (!indices || !data))
    return fail(c, SGV_ERR_ARG, "sgv_set_ld_block_csr: %lld entries without indices/data",
                (long long)indptr[n]);
  if (indptr[0] != 0) return fail(c, SGV_ERR_ARG, "sgv_set_ld_block_csr: indptr[0] != 0");
  int64_t bw = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (indptr[i + 1] < indptr[i])
      return fail(c, SGV_ERR_ARG, "sgv_set_ld_block_csr: indptr decreases at row %lld",
                  (long long)i);
    for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) {
      const int64_t j = indices[e];
      if (j < i || j >= n)
        return fail(c, SGV_ERR_ARG,
                    "sgv_set_ld_block_csr: entry (%lld, %lld) outside the upper triangle of a "
                    "%lld-marker block", (long long)i, (long long)j, (long long)n);
      bw = std::max(bw, j - i);
    }
  }
  int64_t ext = round_up(SYM_H + bw, BAND_Q);
  if (ext >= n) ext = 0;   // the band is as wide as the triangle
  CHK(ld_alloc(c, ld, b, 1, ext));
  const LdBlock& lb = c->ldb[ld][b];
  size_t pmax = 0;
  for (size_t g = 0; g < lb.poff.size(); ++g) pmax = std::max<size_t>(pmax, SYM_H * lb.pw[g]);
  CHK(ensure_hstage(c, sizeof(double) * pmax));
  double* hp = (double*)c->h_stage;
  for (size_t g = 0; g < lb.poff.size(); ++g) {
    const int64_t r0 = (int64_t)g * SYM_H, H = std::min<int64_t>(SYM_H, n - r0);
    const int64_t w = lb.pw[g];
    std::memset(hp, 0, sizeof(double) * (size_t)(H * w));
    for (int64_t i = r0; i < r0 + H; ++i)
      for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) hp[(i - r0) * w + (indices[e] - r0)] += data[e];
    for (int64_t a = 0; a < H; ++a)   // the panel's diagonal block is stored in full
      for (int64_t d = a + 1; d < H; ++d) hp[d * w + a] = hp[a * w + d];
    HIPCHK(hipMemcpyAsync(lb.ptr + lb.poff[g], hp, sizeof(double) * (size_t)(H * w),
                          hipMemcpyHostToDevice, c->st));
    CHK(stream_wait(c));   // the pinned panel buffer is reused
  }
  std::fill(c->rx0_valid.begin(), c->rx0_valid.end(), 0);
  return SGV_OK;
}

extern "C" int sgv_get_ld_block(sgv_ctx* c, int ld, int b, double* host, int64_t ld_host) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || b < 0 || b >= c->nblk || !host || ld_host < c->bn[b])
    return fail(c, SGV_ERR_ARG, "sgv_get_ld_block: bad arguments (ld=%d b=%d)", ld, b);
  CHK(ld_ready(c, ld));
  const int64_t n = c->bn[b];
  const LdBlock& lb = c->ldb[ld][b];
  CHK(stream_wait(c));
  if (lb.fmt == 0) {
    HIPCHK(hipMemcpy2D(host, sizeof(double) * ld_host, lb.ptr, sizeof(double) * c->lda[b],
                       sizeof(double) * n, n, hipMemcpyDeviceToHost));
    return SGV_OK;
  }
  if (lb.ext > 0)   // outside the band nothing is stored
    for (int64_t i = 0; i < n; ++i) std::memset(host + i * ld_host, 0, sizeof(double) * n);
  for (size_t g = 0; g < lb.poff.size(); ++g) {
    const int64_t r0 = (int64_t)g * SYM_H, H = std::min<int64_t>(SYM_H, n - r0);
    HIPCHK(hipMemcpy2D(host + r0 * ld_host + r0, sizeof(double) * ld_host, lb.ptr + lb.poff[g],
                       sizeof(double) * lb.pw[g], sizeof(double) * panel_ext(n, r0, lb.ext), H,
                       hipMemcpyDeviceToHost));
  }
  for (int64_t i = 0; i < n; ++i) {          // mirror the part left of each panel
    const int64_t r0 = (i / SYM_H) * SYM_H;
    for (int64_t j = 0; j < r0; ++j) host[i * ld_host + j] = host[j * ld_host + i];
  }
  return SGV_OK;
}

extern "C" int sgv_ld_block_format(sgv_ctx* c, int ld, int b, int* fmt_out) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || b < 0 || b >= c->nblk || !fmt_out)
    return fail(c, SGV_ERR_ARG, "sgv_ld_block_format: bad arguments");
  const LdBlock& lb = c->ldb[ld][b];
  *fmt_out = lb.ptr ? (lb.fmt == 1 && lb.ext > 0 ? 2 : lb.fmt) : -1;
  return SGV_OK;
}

extern "C" int sgv_set_ld_coupling(sgv_ctx* c, int ld, int gb, int nr, int nc, const double* C) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || gb < 0 || gb + 1 >= c->nblk_global || nr < 1 || nc < 1)
    return fail(c, SGV_ERR_ARG, "sgv_set_ld_coupling: bad arguments (ld %d, gb %d, %d x %d)", ld,
                gb, nr, nc);
  const int ba = gb - c->blk0, bb = gb + 1 - c->blk0;
  const bool la = ba >= 0 && ba < c->nblk, lb = bb >= 0 && bb < c->nblk;
  if ((la && nr > c->bn[ba]) || (lb && nc > c->bn[bb]))
    return fail(c, SGV_ERR_ARG, "sgv_set_ld_coupling: %d x %d exceeds the pieces", nr, nc);
  if ((la || lb) && !C) return fail(c, SGV_ERR_ARG, "sgv_set_ld_coupling: C is null");
  std::vector<LdCoupling>& cv = c->cpl[ld];
  auto it = std::find_if(cv.begin(), cv.end(), [&](const LdCoupling& q) { return q.gb == gb; });
  if (it == cv.end()) {
    cv.push_back(LdCoupling());
    it = cv.end() - 1;
  }
  if (it->d_up) HIPCHK(hipFree(it->d_up));
  if (it->d_lo) HIPCHK(hipFree(it->d_lo));
  it->d_up = it->d_lo = nullptr;
  it->gb = gb;
  it->nr = nr;
  it->nc = nc;
  const size_t n = (size_t)nr * nc;
  if (la) {   // C^T, for gb's tail rows
    std::vector<double> t(n);
    for (int i = 0; i < nr; ++i)
      for (int j = 0; j < nc; ++j) t[(size_t)j * nr + i] = C[(size_t)i * nc + j];
    HIPCHK(hipMalloc(&it->d_up, sizeof(double) * n));
    HIPCHK(hipMemcpy(it->d_up, t.data(), sizeof(double) * n, hipMemcpyHostToDevice));
  }
  if (lb) {   // C, for gb + 1's head rows
    HIPCHK(hipMalloc(&it->d_lo, sizeof(double) * n));
    HIPCHK(hipMemcpy(it->d_lo, C, sizeof(double) * n, hipMemcpyHostToDevice));
  }
  std::sort(cv.begin(), cv.end(), [](const LdCoupling& a, const LdCoupling& b) { return a.gb < b.gb; });
  c->plan[ld].valid = false;
  return SGV_OK;
}

extern "C" int sgv_ld_stored_bytes(sgv_ctx* c, int ld, double* out) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || !out) return fail(c, SGV_ERR_ARG, "sgv_ld_stored_bytes: bad arguments");
  double s = 0.0;
  for (int b = 0; b < c->nblk; ++b)
    if (c->ldb[ld][b].ptr) s += c->ldb[ld][b].stored_bytes;
  *out = s;
  return SGV_OK;
}

extern "C" int sgv_set_ridge(sgv_ctx* c, double s) {
  ENTER(c);
  c->s = s;
  std::fill(c->rx0_valid.begin(), c->rx0_valid.end(), 0);
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
// denoiser (src/sgvamp.py:93-114, 270-291)
// ---------------------------------------------------------------------------
// denoiser kernel + the ordered reduction of its derivative sums into h_tot[0..K);
// metrics: the four metrics sums of the new xhat1 (sgv_metrics) in the same
// reduction, h_tot[K .. K + 3] (one exchange instead of two with a communicator;
// not with more than MAXK cohorts) -- returns whether they were fused
static int denoise_enqueue(sgv_ctx* c, const double* gam1s, const double* a, double lam,
                           int nslab, const double* omegas, const double* sigmas, double rho,
                           int damp, bool metrics = false, bool* fused = nullptr) {
  DenoiseArgs da{};
  da.xhat1 = c->xhat1;
  da.nslab = nslab;
  da.lam = lam;
  da.rho = rho;
  da.damp = damp;
  da.write_x = 1;
  for (int k = 0; k < c->K; ++k) {
    const double ag = a[k] * gam1s[k];                 // self.a * gam1s
    da.sum_ag = (k == 0) ? ag : da.sum_ag + ag;        // builtin sum (:95)
  }
  for (int l = 0; l < nslab; ++l) {
    da.omegas[l] = omegas[l];
    da.sigmas[l] = sigmas[l];
    da.s2[l] = 1.0 / (da.sum_ag + 1.0 / sigmas[l]);     // :95
    da.sq[l] = std::sqrt(da.s2[l] / sigmas[l]);         // np.sqrt(sigma2_meta / sigmas)
  }
  // more than MAXK cohorts: groups of MAXK.  np.inner over all of them first
  // (one sequential sum continued group to group), then one launch per group
  // for its cohorts' derivative sums; the first also writes xhat1
  const int ng = (c->K + MAXK - 1) / MAXK;
  auto group = [&](int g) {
    da.K = std::min(MAXK, c->K - g * MAXK);
    for (int k = 0; k < da.K; ++k) {
      const int kk = g * MAXK + k;
      da.r1[k] = c->r1[kk];
      da.a[k] = a[kk];
      da.gam1[k] = gam1s[kk];
      da.ag[k] = a[kk] * gam1s[kk];
    }
  };
  if (ng > 1) {
    CHK(grow(c, &c->d_inner, &c->inner_cap, (size_t)std::max<int64_t>(c->Mpad, 1)));
    for (int g = 0; g < ng; ++g) {
      group(g);
      HIPCHK(launch_den_inner(c->d_ch, c->nch, da, c->d_inner, g == 0 ? 1 : 0, c->st));
    }
    da.inner = c->d_inner;
  }
  const bool met = metrics && ng == 1;
  if (fused) *fused = met;
  for (int g = 0; g < ng; ++g) {
    group(g);
    da.write_x = g == 0 ? 1 : 0;
    da.x0 = met ? c->x0 : nullptr;
    HIPCHK(launch_denoise(c->d_ch, c->nch, da, c->d_part, c->st));
    CHK(reduce_dev(c, da.K + (met ? 4 : 0), c->d_ch_begin, identity_map(), c->h_tot + g * MAXK));
  }
  return SGV_OK;
}

extern "C" int sgv_denoise(sgv_ctx* c, const double* gam1s, const double* a, double lam,
                           int nslab, const double* omegas, const double* sigmas, double rho,
                           int damp, double* der_sum) {
  ENTER(c);
  if (nslab < 1 || nslab > MAXL || !gam1s || !a || !omegas || !sigmas || !der_sum)
    return fail(c, SGV_ERR_ARG, "sgv_denoise: bad arguments (nslab=%d)", nslab);
  CHK(denoise_enqueue(c, gam1s, a, lam, nslab, omegas, sigmas, rho, damp));
  CHK(stream_wait(c));
  resolve_timers(c);
  for (int k = 0; k < c->K; ++k) der_sum[k] = c->h_tot[k];
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// EM prior loop (src/sgvamp.py:116-136, 250-257)
// ---------------------------------------------------------------------------
extern "C" int sgv_em(sgv_ctx* c, const double* gam1s, const double* a, int nslab,
                      const double* sigmas, int maxit, double* lam_io, double* omegas_io,
                      int* steps_out, double* final_err_out) {
  ENTER(c);
  if (nslab < 1 || nslab > MAXL || !gam1s || !a || !sigmas || !lam_io || !omegas_io)
    return fail(c, SGV_ERR_ARG, "sgv_em: bad arguments");
  // more than MAXK cohorts: one k_em launch per group of MAXK, the later ones
  // adding to the first's partials (each marker's cohort sum then runs group
  // by group); np.average's weight sum covers all cohorts
  const int ngr = (c->K + MAXK - 1) / MAXK;
  std::vector<EmArgs> eg(ngr);
  EmArgs& ea = eg[0];
  double scl = 0.0;
  for (int k = 0; k < c->K; ++k) scl = (k == 0) ? a[0] : scl + a[k];
  for (int g = 0; g < ngr; ++g) {
    EmArgs& e = eg[g];
    e = EmArgs{};
    e.K = std::min(MAXK, c->K - g * MAXK);
    e.nslab = nslab;
    for (int k = 0; k < e.K; ++k) {
      e.r1[k] = c->r1[g * MAXK + k];
      e.a[k] = a[g * MAXK + k];
      e.gam1[k] = gam1s[g * MAXK + k];
    }
    e.scl = scl;
    e.accum = g > 0 ? 1 : 0;
    for (int l = 0; l < nslab; ++l) e.sigmas[l] = sigmas[l];
    e.tab = c->d_emtab + (size_t)g * MAXK * EM_TAB;
    HIPCHK(launch_em_prep(e, c->d_emtab + (size_t)g * MAXK * EM_TAB, c->st));
  }
  auto em_groups = [&](const ChunkDesc* ch, int nch, double* part) -> int {
    for (int g = 0; g < ngr; ++g) HIPCHK(launch_em(ch, nch, eg[g], part, c->st));
    return SGV_OK;
  };
  double lam = *lam_io;
  double om[MAXL];
  for (int l = 0; l < nslab; ++l) om[l] = omegas_io[l];
  if (c->cg_pipe && maxit > 0) {
    // Device loop: k_em reads lam/omegas from the device state, k_em_ctl updates
    // it and tests convergence; step it + 1 is enqueued before the host waits
    // for step it's test, so the GPU does not idle for a host round trip per
    // step (one no-op step runs past the last).  Every rank enqueues the same
    // steps (the stop decision is made from the same global sums).
    EmState* hi = c->h_emi;   // the previous loop's init copy has completed
    std::memset(hi, 0, sizeof(EmState));
    hi->lam = lam;
    for (int l = 0; l < nslab; ++l) hi->om[l] = om[l];
    HIPCHK(hipMemcpyAsync(c->d_ems, hi, sizeof(EmState), hipMemcpyHostToDevice, c->st));
    for (EmArgs& e : eg) e.st = c->d_ems;
    // one rank: reduction + control in one launch (k_em_reduce_ctl, same bits).
    // With a communicator: the replicated EM (em_rep_setup) runs the same
    // one-rank loop over every rank's gathered r1.
    const bool rep = em_mode_pick(c, maxit);
    const bool fuse = rep || (!c->comm && !c->host_ag && fused_ctl_pays(EM_NV, c->nblk));
    const ChunkDesc* ech = rep ? c->d_chg : c->d_ch;
    const int* ebeg = rep ? c->d_chg_begin : c->d_ch_begin;
    const int enb = rep ? c->nblkg : c->nblk, ench = rep ? c->nchg : c->nch;
    double* epart = rep ? c->d_partg : c->d_part;
    if (rep) {
      CHK(gather_r1(c));
      for (int k = 0; k < c->K; ++k) ea.r1[k] = c->d_r1g + (size_t)k * c->mpad_max;
    }
    auto enqueue = [&](int j) -> int {
      if (fuse) {
        CHK(em_groups(ech, ench, epart));
        const EmCtl f{ebeg, enb, nslab, c->h_emm + j % CG_RING, (double)c->Mtot, j, maxit};
        HIPCHK(launch_em_reduce_ctl(epart, c->d_ems, f, c->st));
        HIPCHK(hipEventRecord(c->ev_em[j % CG_RING], c->st));
        return SGV_OK;
      }
      CHK(em_groups(c->d_ch, c->nch, c->d_part));
      CHK(reduce_dev(c, EM_NV, c->d_ch_begin, identity_map(), c->d_emtot));
      HIPCHK(launch_em_ctl(c->d_ems, c->h_emm + j % CG_RING, c->d_emtot, nslab, (double)c->Mtot,
                           j, maxit, c->st));
      HIPCHK(hipEventRecord(c->ev_em[j % CG_RING], c->st));
      return SGV_OK;
    };
    CHK(enqueue(0));
    const volatile EmState* last = nullptr;
    for (int it = 0; it < maxit; ++it) {
      if (it + 1 < maxit) CHK(enqueue(it + 1));
      CHK(event_spin(c, c->ev_em[it % CG_RING]));
      last = c->h_emm + it % CG_RING;
      if (last->done) break;
    }
    *lam_io = last->lam;
    for (int l = 0; l < nslab; ++l) omegas_io[l] = last->om[l];
    if (steps_out) *steps_out = last->steps;
    if (final_err_out) *final_err_out = last->err;
    c->em_prev_steps = last->steps;   // the same on every rank
    return SGV_OK;
  }
  double om_err = 0.0, lam_err = 0.0;
  int steps = 0;
  for (int it = 0; it < maxit; ++it) {
    for (EmArgs& e : eg) {
      e.lam = lam;
      for (int l = 0; l < nslab; ++l) e.omegas[l] = om[l];
    }
    CHK(em_groups(c->d_ch, c->nch, c->d_part));
    double tot[EM_NV];
    CHK(reduce_host(c, EM_NV, c->d_ch_begin, tot));
    const double lam_new = tot[0] / (double)c->Mtot;   // np.mean (:134)
    double om_new[MAXL];
    double dn = 0.0, on = 0.0;
    for (int l = 0; l < nslab; ++l) {
      om_new[l] = tot[1 + l] / tot[1 + nslab];         // :136
      const double d = om_new[l] - om[l];
      dn += d * d;
      on += om[l] * om[l];
    }
    om_err = std::sqrt(dn) / std::sqrt(on);            // :254
    lam_err = std::fabs(lam_new - lam) / lam_new;      // :255
    lam = lam_new;
    for (int l = 0; l < nslab; ++l) om[l] = om_new[l];
    steps = it + 1;
    if (om_err < 1e-6 && lam_err < 1e-6) break;        // :256
  }
  *lam_io = lam;
  for (int l = 0; l < nslab; ++l) omegas_io[l] = om[l];
  if (steps_out) *steps_out = steps;
  if (final_err_out) *final_err_out = std::max(om_err, lam_err);
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// LMMSE (src/sgvamp.py:301-364)
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// MLE prior update (src/sgvamp.py:139-194): the K x M x L sums of
// Lagrangian_der on the device; fsolve (MINPACK hybrd) stays on the host
// ---------------------------------------------------------------------------
// cohort group g (MAXK cohorts from g * MAXK)
static int mle_args(sgv_ctx* c, const double* gam1s, int L, const double* sigma2, int g,
                    MleArgs* m) {
  if (!gam1s || !sigma2 || L < 1 || L > MAXL + 1) return fail(c, SGV_ERR_ARG, "bad MLE arguments");
  *m = MleArgs{};
  m->K = std::min(MAXK, c->K - g * MAXK);
  m->L = L;
  for (int k = 0; k < m->K; ++k) {
    m->r1[k] = c->r1[g * MAXK + k];
    m->ginv[k] = 1.0 / gam1s[g * MAXK + k];                 // :146
  }
  for (int l = 0; l < L; ++l) m->sigma2[l] = sigma2[l];
  return SGV_OK;
}

extern "C" int sgv_mle_exp_max(sgv_ctx* c, const double* gam1s, int L, const double* sigma2,
                               double* exp_max) {
  ENTER(c);
  if (!exp_max) return fail(c, SGV_ERR_ARG, "exp_max is null");
  // :152: max over (k, m, l) of (-r1^2 / 2) / v_kl, attained at min_m r1_km^2
  double best = -std::numeric_limits<double>::infinity();
  for (int g = 0; g * MAXK < c->K; ++g) {
    MleArgs m;
    CHK(mle_args(c, gam1s, L, sigma2, g, &m));
    HIPCHK(launch_mle_minsq(c->d_ch, c->nch, m, c->d_part, c->st));
    double mn[MAXK];
    CHK(reduce_host(c, MAXK, c->d_ch_begin, mn, /*op=min*/ 1));
    for (int k = 0; k < m.K; ++k)
      for (int l = 0; l < L; ++l) best = std::max(best, -mn[k] / 2.0 / (m.sigma2[l] + m.ginv[k]));
  }
  *exp_max = best;
  return SGV_OK;
}

extern "C" int sgv_mle_terms(sgv_ctx* c, const double* a, const double* gam1s, int L,
                             const double* sigma2, const double* omega, double exp_max,
                             double* sums) {
  ENTER(c);
  if (!a || !omega || !sums) return fail(c, SGV_ERR_ARG, "bad MLE arguments");
  // one launch per cohort group; the groups' totals are added in group order
  for (int g = 0; g * MAXK < c->K; ++g) {
    MleArgs m;
    CHK(mle_args(c, gam1s, L, sigma2, g, &m));
    for (int k = 0; k < m.K; ++k) m.a[k] = a[g * MAXK + k];
    for (int l = 0; l < L; ++l) m.omega[l] = omega[l];
    m.exp_max = exp_max;
    HIPCHK(launch_mle_terms(c->d_ch, c->nch, m, c->d_part, c->st));
    double tot[MAXL + 1];
    CHK(reduce_host(c, MAXL + 1, c->d_ch_begin, tot));
    for (int l = 0; l < L; ++l) sums[l] = g == 0 ? tot[l] : sums[l] + tot[l];
  }
  return SGV_OK;
}

// The MLE prior update, src/sgvamp.py:162-194, with scipy's fsolve restated in
// hybrd.cpp; each function evaluation is one device pass over the r1 vectors
// (sgv_mle_terms), the rest the reference's host arithmetic in its order.
struct MleFn {
  sgv_ctx* c;
  const double* gam1s;
  const double* a;
  int L;
  const double* sigma2;
  const double* omega0;
  double exp_max;
  int rc;
  // the sums of the last evaluation and the omega they were taken at: the
  // Jacobian's gam column (x[L] perturbed) has the same omega, so its sums are
  // these, bitwise (the device sums are deterministic)
  double S[MAXL + 1], Sx[MAXL + 1];
  bool have_s;
};

// Lagrangian_der (:159-160) from the sums S at omega = x[:L]
static void mle_residual(const MleFn& f, const double* x, const double* S, double* y) {
  const int L = f.L;
  const double gam = x[L];
  for (int l = 0; l < L; ++l) y[l] = (S[l] + (f.omega0[l] - 1.0) / x[l]) + gam;   // :159
  double sw = 0.0;                                                                   // :160
  for (int l = 0; l < L; ++l) sw += x[l];
  y[L] = sw - 1.0;
}

static int mle_lagrangian(void* user, int n, const double* x, double* y) {
  MleFn& f = *(MleFn*)user;
  const int L = f.L;
  f.rc = sgv_mle_terms(f.c, f.a, f.gam1s, L, f.sigma2, x, f.exp_max, f.S);   // omega = x[:L]
  if (f.rc != SGV_OK) return -1;
  std::memcpy(f.Sx, x, sizeof(double) * L);
  f.have_s = true;
  mle_residual(f, x, f.S, y);
  (void)n;
  return 0;
}

// the forward-difference Jacobian's n = L + 1 points (hybrd's fdjac1): the L
// omega columns' device sums enqueued back to back with one host wait instead
// of one per point, the gam column from the base point's sums.  One cohort
// group, one rank (the host exchange waits per reduction anyway); otherwise
// point by point.  Each point's sums are the same launches as mle_lagrangian's,
// so the Jacobian is bitwise the per-point one.
static int mle_jacobian(void* user, int n, const double* x, const double* h, double* F) {
  MleFn& f = *(MleFn*)user;
  sgv_ctx* c = f.c;
  const int L = f.L;
  double xj[MAXL + 2];
  const bool base = f.have_s && std::memcmp(f.Sx, x, sizeof(double) * L) == 0;
  if (c->K > MAXK || c->comm || c->host_ag) {
    for (int j = 0; j < n; ++j) {
      std::memcpy(xj, x, sizeof(double) * n);
      xj[j] = x[j] + h[j];
      if (mle_lagrangian(user, n, xj, F + (size_t)j * n) < 0) return -1;
    }
    return 0;
  }
  f.rc = [&]() -> int {
    ENTER(c);
    MleArgs m;
    CHK(mle_args(c, f.gam1s, L, f.sigma2, 0, &m));
    for (int k = 0; k < m.K; ++k) m.a[k] = f.a[k];
    m.exp_max = f.exp_max;
    for (int j = 0; j < L; ++j) {
      for (int l = 0; l < L; ++l) m.omega[l] = l == j ? x[l] + h[l] : x[l];
      HIPCHK(launch_mle_terms(c->d_ch, c->nch, m, c->d_part, c->st));
      CHK(reduce_dev(c, MAXL + 1, c->d_ch_begin, identity_map(), c->h_tot + j * (MAXL + 1)));
    }
    CHK(stream_wait(c));
    resolve_timers(c);
    return SGV_OK;
  }();
  if (f.rc != SGV_OK) return -1;
  double base_s[MAXL + 1];
  if (base) std::memcpy(base_s, f.S, sizeof(double) * L);
  for (int j = 0; j < L; ++j) {
    std::memcpy(xj, x, sizeof(double) * n);
    xj[j] = x[j] + h[j];
    std::memcpy(f.S, c->h_tot + j * (MAXL + 1), sizeof(double) * L);
    std::memcpy(f.Sx, xj, sizeof(double) * L);
    mle_residual(f, xj, f.S, F + (size_t)j * n);
  }
  // the gam column: omega = x[:L], the base point's sums
  std::memcpy(xj, x, sizeof(double) * n);
  xj[L] = x[L] + h[L];
  if (base) {
    std::memcpy(f.S, base_s, sizeof(double) * L);
    std::memcpy(f.Sx, x, sizeof(double) * L);
    mle_residual(f, xj, f.S, F + (size_t)L * n);
    return 0;
  }
  return mle_lagrangian(user, n, xj, F + (size_t)L * n);
}

extern "C" int sgv_mle_update(sgv_ctx* c, const double* gam1s, const double* a, int nslab,
                              const double* sigmas, double* lam_io, double* omegas_io,
                              double* gam_io, int* status_out) {
  ENTER(c);
  if (!gam1s || !a || !sigmas || !lam_io || !omegas_io || !gam_io || !status_out ||
      nslab < 1 || nslab > MAXL)
    return fail(c, SGV_ERR_ARG, "sgv_mle_update: bad arguments");
  const int L = nslab + 1;
  double omega0[MAXL + 1], sigma2[MAXL + 1], x[MAXL + 2];
  omega0[0] = 1 - *lam_io;                                        // :166-168
  for (int l = 0; l < nslab; ++l) omega0[1 + l] = *lam_io * omegas_io[l];
  sigma2[0] = 1e-16;                                              // :169-171
  for (int l = 0; l < nslab; ++l) sigma2[1 + l] = sigmas[l];
  for (int l = 0; l < L; ++l) x[l] = omega0[l];                   // :173-178
  x[L] = std::isnan(*gam_io) ? 1.0 : *gam_io;
  MleFn f{c, gam1s, a, L, sigma2, omega0, 0.0, SGV_OK, {}, {}, false};
  CHK(sgv_mle_exp_max(c, gam1s, L, sigma2, &f.exp_max));           // :152, once per update
  // :179 (the forward-difference Jacobian's points batched, mle_jacobian)
  const int ier = sgv_fsolve_jac(L + 1, mle_lagrangian, mle_jacobian, &f, x, nullptr, nullptr);
  if (f.rc != SGV_OK) return f.rc;
  if (ier != 1) {                                                 // :181-184
    *status_out = SGV_MLE_NOT_CONVERGED;
    return SGV_OK;
  }
  for (int l = 0; l < L; ++l)
    if (x[l] <= 0) {                                              // :185-188
      *status_out = SGV_MLE_NEGATIVE;
      return SGV_OK;
    }
  double sw = 0.0;                                                // :190 x[:-1] /= sum(x[:-1])
  for (int l = 0; l < L; ++l) sw += x[l];
  for (int l = 0; l < L; ++l) x[l] = x[l] / sw;
  *lam_io = 1 - x[0];                                             // :191
  double ss = 0.0;                                                // :192 w / sum(x[1:-1])
  for (int l = 1; l < L; ++l) ss += x[l];
  for (int l = 0; l < nslab; ++l) omegas_io[l] = x[1 + l] / ss;
  *gam_io = x[L];                                                 // :193
  *status_out = 0;
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

// LMMSE of the cohorts g0 .. g0 + Kg - 1 (Kg <= MAXKG: 2 Kg <= MAXC CG columns,
// one batched CG loop); per-cohort inputs/outputs are the group's slices
static int lmmse_group(sgv_ctx* c, int g0, int Kg, const double* gamw, const double* gam2,
                       const double* alpha1, const double* alpha2_prev, int cg_maxit, double rtol,
                       int lmmse_damp, double rho, int learn_gamw, double* out, int* cg_out,
                       int* passes_out) {
  const int K = Kg, ncol = 2 * K;
  const double s = c->s;
  int passes = 0;

  // warm start needs R_s x0: carried from the previous iteration (rs_rec), or the
  // previous gamw pass; a pass only when X was set from outside
  for (int ld = 0; ld < c->nld; ++ld) {
    PassArgs pa{};
    int nc = 0;
    for (int j = 0; j < ncol; ++j) {
      if (!c->xnz[2 * g0 + j] || c->rx0_valid[2 * g0 + j] || c->ld_of[g0 + (j / 2)] != ld) continue;
      pa.in[nc] = c->X[2 * g0 + j];
      pa.out[nc] = c->RX0[2 * g0 + j];
      pa.dot[nc] = nullptr;
      pa.c1[nc] = 1.0 - s;
      pa.c2[nc] = s;
      ++nc;
      c->rx0_valid[2 * g0 + j] = 1;
    }
    if (nc) {
      CHK(ld_pass(c, ld, nc, pa));
      ++passes;
    }
  }

  // r2, mu2, r0 = b - A x0, p0 = r0 (:305-313, iterative.py:376-392)
  InitArgs ia{};
  ia.xhat1 = c->xhat1;
  ia.K = K;
  ia.save_x0 = lmmse_damp;
  for (int k = 0; k < K; ++k) {
    ia.cp.r[k] = c->r[g0 + k];
    ia.cp.r1[k] = c->r1[g0 + k];
    ia.cp.r2[k] = c->r2[g0 + k];
    ia.cp.u[k] = c->U[g0 + k];
    ia.alpha1[k] = alpha1[k];
    ia.gamw[k] = gamw[k];
    ia.gam2[k] = gam2[k];
  }
  for (int j = 0; j < ncol; ++j) {
    ia.col.X[j] = c->X[2 * g0 + j];
    ia.col.X0[j] = c->X0[2 * g0 + j];
    ia.col.Rr[j] = c->Rr[2 * g0 + j];
    ia.col.P[j] = c->P[2 * g0 + j];
    ia.col.Q[j] = c->Q[2 * g0 + j];
    ia.col.RX0[j] = c->RX0[2 * g0 + j];
    ia.col.RXp[j] = c->rs_rec ? c->RXp[2 * g0 + j] : nullptr;
    ia.warm[j] = c->xnz[2 * g0 + j];
  }
  double tot[2 * MAXC];
  const bool dev_init = c->cg_pipe;   // CG prologue on the device: no host round trip
  // with a communicator and one LD matrix for the group's columns: the prologue's
  // sums share iteration 0's exchange (cg_loop_dev, CgMerge0)
  bool one_ld = true;
  for (int k = 1; k < K; ++k) one_ld &= c->ld_of[g0 + k] == c->ld_of[g0];
  const bool merge0 = dev_init && (c->comm || c->host_ag) && one_ld;
  if (merge0) CHK(grow(c, &c->d_part2, &c->part2_cap, (size_t)c->nch * 2 * MAXC));
  HIPCHK(launch_lmmse_init(c->d_ch, c->nch, ia, merge0 ? c->d_part2 : c->d_part, c->st));
  CgMerge0 mg;
  if (merge0) {
    mg.part = c->d_part2;
    mg.rtol = rtol;
    mg.X = c->X.data() + 2 * g0;
    mg.RX = c->RX0.data() + 2 * g0;
  } else if (dev_init) {
    CHK(reduce_dev(c, 2 * MAXC, c->d_ch_begin, identity_map(), c->d_tot));
    HIPCHK(launch_cg_init(c->d_cgs, c->d_tot, rtol, ncol, c->d_ch, c->nch, c->X.data() + 2 * g0,
                          c->RX0.data() + 2 * g0, c->st));
  } else {
    CHK(reduce_host(c, 2 * MAXC, c->d_ch_begin, tot));
  }
  // carried: RX0 follows X through the CG; otherwise the gamw pass refreshes it
  for (int j = 0; j < ncol; ++j) c->rx0_valid[2 * g0 + j] = c->rs_rec ? 1 : 0;

  CgCols cc;
  cc.ncol = ncol;
  double rhov[MAXC], atol[MAXC];
  int active[MAXC], iters[MAXC], info[MAXC];
  for (int j = 0; j < ncol; ++j) {
    const int k = j / 2;
    cc.col_ld[j] = c->ld_of[g0 + k];
    cc.c1[j] = gamw[k] * (1.0 - s);           // A = gamw R_s + gam2 I (:312)
    cc.c2[j] = gamw[k] * s + gam2[k];
    cc.X[j] = c->X[2 * g0 + j];
    cc.Rr[j] = c->Rr[2 * g0 + j];
    cc.P[j] = c->P[2 * g0 + j];
    cc.Q[j] = c->Q[2 * g0 + j];
    if (c->rs_rec) {
      cc.RX[j] = c->RX0[2 * g0 + j];
      cc.Y[j] = c->Y[2 * g0 + j];
    }
    active[j] = 1;
    if (dev_init) continue;                   // k_cg_init
    const double bn = std::sqrt(tot[j]);      // bnrm2 (iterative.py:376)
    atol[j] = std::max(0.0, rtol * bn);
    rhov[j] = tot[MAXC + j];
    if (bn == 0.0) {                          // iterative.py:380-381: return b
      HIPCHK(hipMemsetAsync(c->X[2 * g0 + j], 0, sizeof(double) * c->Mpad, c->st));
      HIPCHK(hipMemsetAsync(c->RX0[2 * g0 + j], 0, sizeof(double) * c->Mpad, c->st));   // R_s 0
      active[j] = 0;
    }
  }
  cc.s = s;
  CHK(dev_init ? cg_loop_dev(c, cc, nullptr, nullptr, cg_maxit, active, iters, info, &passes,
                             merge0 ? &mg : nullptr)
               : cg_run(c, cc, rhov, atol, cg_maxit, active, iters, info, &passes));

  // damping, u.Sigma2_u, xhat2.r, x.any() (:322-323, 338, 352)
  PostArgs po{};
  po.K = K;
  po.damp = lmmse_damp;
  po.rs = c->rs_rec;
  po.rho = rho;
  for (int j = 0; j < ncol; ++j) {
    po.X[j] = c->X[2 * g0 + j];
    po.X0[j] = c->X0[2 * g0 + j];
    po.RX[j] = c->RX0[2 * g0 + j];
    po.RXp[j] = c->RXp[2 * g0 + j];
  }
  for (int k = 0; k < K; ++k) {
    po.u[k] = c->U[g0 + k];
    po.r[k] = c->r[g0 + k];
  }
  HIPCHK(launch_lmmse_post(c->d_ch, c->nch, po, c->d_part, c->st));
  double pt[4 * MAXKG + MAXC];
  R1Args ra{};
  ra.K = K;
  if (dev_init) {
    // r1 takes alpha2 from the device-reduced Tr(Sigma2): the update is queued
    // before the host reads the sums (which it computes alpha2 from as well)
    CHK(reduce_dev(c, 4 * MAXKG + MAXC, c->d_ch_begin, identity_map(), c->d_tot));
    ra.trs = c->d_tot;
    ra.Mtot = (double)c->Mtot;
    ra.rho = rho;
    ra.damp = lmmse_damp;
    for (int k = 0; k < K; ++k) {
      ra.X[k] = c->X[2 * g0 + (2 * k)];
      ra.r2[k] = c->r2[g0 + k];
      ra.r1[k] = c->r1[g0 + k];
      ra.gam2[k] = gam2[k];
      ra.alpha2_prev[k] = alpha2_prev[k];
    }
    HIPCHK(launch_r1_update(c->d_ch, c->nch, ra, c->st));   // :348
    HIPCHK(launch_copy_f64(c->h_tot, c->d_tot, 4 * MAXKG + MAXC, c->st));
    CHK(stream_wait(c));
    resolve_timers(c);
    std::memcpy(pt, c->h_tot, sizeof(pt));
  } else {
    CHK(reduce_host(c, 4 * MAXKG + MAXC, c->d_ch_begin, pt));
  }
  for (int j = 0; j < ncol; ++j) c->xnz[2 * g0 + j] = pt[2 * MAXKG + j] > 0.0;

  for (int k = 0; k < K; ++k) {
    const double TrSigma2 = pt[k];
    double a2 = gam2[k] * TrSigma2 / (double)c->Mtot;              // :340
    if (lmmse_damp) a2 = rho * a2 + (1 - rho) * alpha2_prev[k];    // :345-346
    const double g1 = gam2[k] * (1 - a2) / a2;                    // :347
    double* o = out + (size_t)k * SGV_LMMSE_NOUT;
    o[SGV_O_TRSIGMA2] = TrSigma2;
    o[SGV_O_ALPHA2] = a2;
    o[SGV_O_GAM1] = g1;
    o[SGV_O_XR] = pt[MAXKG + k];
    o[SGV_O_Z] = 0.0;
    o[SGV_O_TRRSIGMA2] = 0.0;
    o[SGV_O_XRX] = 0.0;
    o[SGV_O_GAMW] = gamw[k];
    ra.X[k] = c->X[2 * g0 + (2 * k)];
    ra.r2[k] = c->r2[g0 + k];
    ra.r1[k] = c->r1[g0 + k];
    ra.alpha2[k] = a2;
    cg_out[4 * k + 0] = iters[2 * k];
    cg_out[4 * k + 1] = info[2 * k];
    cg_out[4 * k + 2] = iters[2 * k + 1];
    cg_out[4 * k + 3] = info[2 * k + 1];
  }
  if (!dev_init) HIPCHK(launch_r1_update(c->d_ch, c->nch, ra, c->st));   // :348

  if (learn_gamw && c->rs_rec) {  // :350-363 from the carried products: no pass
    for (int k = 0; k < K; ++k) {
      const double N = c->Ncoh[g0 + k];
      double* o = out + (size_t)k * SGV_LMMSE_NOUT;
      const double xRx = pt[2 * MAXKG + MAXC + k];
      const double TrRSigma2 = pt[3 * MAXKG + MAXC + k];
      double z = N - 2 * o[SGV_O_XR] + xRx;                        // :352
      if (z < 0) z = 0;                                            // :353-354
      o[SGV_O_Z] = z;
      o[SGV_O_XRX] = xRx;
      o[SGV_O_TRRSIGMA2] = TrRSigma2;
      o[SGV_O_GAMW] = 1 / (z / N + TrRSigma2 / N);                 // :363
    }
  } else if (learn_gamw) {  // :350-363; R_s [xhat2, Sigma2_u] is also the next warm start's R_s x0
    for (int ld = 0; ld < c->nld; ++ld) {
      PassArgs pa{};
      Map16 map = identity_map();
      int nc = 0;
      for (int j = 0; j < ncol; ++j) {
        const int k = j / 2;
        if (c->ld_of[g0 + k] != ld) continue;
        pa.in[nc] = c->X[2 * g0 + j];
        pa.out[nc] = c->RX0[2 * g0 + j];
        pa.dot[nc] = (j % 2 == 0) ? c->X[2 * g0 + j] : c->U[g0 + k];
        pa.c1[nc] = 1.0 - s;
        pa.c2[nc] = s;
        map.d[nc] = j;
        ++nc;
        c->rx0_valid[2 * g0 + j] = 1;
      }
      if (!nc) continue;
      CHK(ld_pass(c, ld, nc, pa));
      ++passes;
      double gt[MAXC];
      CHK(reduce_dev(c, nc, ld_parts(c, ld), map, c->h_tot));
      CHK(stream_wait(c));
      resolve_timers(c);
      std::memcpy(gt, c->h_tot, sizeof(double) * ncol);
      for (int k = 0; k < K; ++k) {
        if (c->ld_of[g0 + k] != ld) continue;
        const double N = c->Ncoh[g0 + k];
        double* o = out + (size_t)k * SGV_LMMSE_NOUT;
        const double xRx = gt[2 * k];
        const double TrRSigma2 = gt[2 * k + 1];
        double z = N - 2 * o[SGV_O_XR] + xRx;                      // :352
        if (z < 0) z = 0;                                          // :353-354
        o[SGV_O_Z] = z;
        o[SGV_O_XRX] = xRx;
        o[SGV_O_TRRSIGMA2] = TrRSigma2;
        o[SGV_O_GAMW] = 1 / (z / N + TrRSigma2 / N);               // :363
      }
    }
  } else {
    CHK(stream_wait(c));
  }
  if (passes_out) *passes_out = passes;
  return SGV_OK;
}

extern "C" int sgv_lmmse(sgv_ctx* c, int it, const double* gamw, const double* gam2,
                         const double* alpha1, const double* alpha2_prev, const int8_t* probes,
                         int cg_maxit, double rtol, int lmmse_damp, double rho, int learn_gamw,
                         double* out, int* cg_out, int* passes_out) {
  ENTER(c);
  (void)it;
  if (!gamw || !gam2 || !alpha1 || !alpha2_prev || !probes || !out || !cg_out || cg_maxit < 0)
    return fail(c, SGV_ERR_ARG, "sgv_lmmse: bad arguments");
  const int K = c->K;

  // probes u_k (:326), int8 +-1 -> f64; uploaded at the start of sgv_step, or now
  int ps = c->pref_slot;
  if (ps < 0 || c->pref_src != probes) CHK(probe_upload(c, probes, &ps));
  c->pref_slot = -1;
  c->pref_src = nullptr;
  HIPCHK(hipStreamWaitEvent(c->st, c->ev_probe[ps], 0));
  for (int k = 0; k < K; ++k)
    HIPCHK(launch_unpack_i8(c->d_ch, c->nch, c->d_ch_doff,
                            c->d_probe + ps * c->probe_cap + (size_t)k * c->Mloc, c->U[k], c->st));
  HIPCHK(hipEventRecord(c->ev_unpk[ps], c->st));

  // cohorts in groups of MAXKG (2 MAXKG = MAXC CG columns per LD pass): the
  // LMMSE of a cohort touches only its own vectors and the shared xhat1, so the
  // groups run one after another with the same per-cohort arithmetic
  int passes = 0;
  for (int g0 = 0; g0 < K; g0 += MAXKG) {
    const int Kg = std::min(MAXKG, K - g0);
    int gp = 0;
    CHK(lmmse_group(c, g0, Kg, gamw + g0, gam2 + g0, alpha1 + g0, alpha2_prev + g0, cg_maxit, rtol,
                    lmmse_damp, rho, learn_gamw, out + (size_t)g0 * SGV_LMMSE_NOUT, cg_out + 4 * g0,
                    &gp));
    passes += gp;
  }
  if (passes_out) *passes_out = passes;
  return SGV_OK;
}

extern "C" int sgv_metrics(sgv_ctx* c, double* out4) {
  ENTER(c);
  if (!out4) return fail(c, SGV_ERR_ARG, "out4 is null");
  HIPCHK(launch_metrics(c->d_ch, c->nch, c->xhat1, c->x0, c->d_part, c->st));
  return reduce_host(c, 4, c->d_ch_begin, out4);
}

// The same sums, queued without a host wait (xhat1 and x0 are not written
// again before sgv_metrics_end); the ordered totals land in pinned memory.
// With the host exchange the reduction itself waits, so begin completes it.
extern "C" int sgv_metrics_begin(sgv_ctx* c) {
  ENTER(c);
  if (!c->h_met) {
    HIPCHK(hipHostMalloc(&c->h_met, sizeof(double) * 4, hipHostMallocCoherent));
    HIPCHK(hipEventCreateWithFlags(&c->ev_met, hipEventDisableTiming));
  }
  HIPCHK(launch_metrics(c->d_ch, c->nch, c->xhat1, c->x0, c->d_part, c->st));
  CHK(reduce_dev(c, 4, c->d_ch_begin, identity_map(), c->h_met));
  HIPCHK(hipEventRecord(c->ev_met, c->st));
  c->met_pending = 1;
  return SGV_OK;
}

extern "C" int sgv_metrics_end(sgv_ctx* c, double* out4) {
  ENTER(c);
  if (!out4) return fail(c, SGV_ERR_ARG, "out4 is null");
  if (!c->met_pending) return fail(c, SGV_ERR_ARG, "sgv_metrics_end without sgv_metrics_begin");
  hipError_t e;
  while ((e = hipEventQuery(c->ev_met)) == hipErrorNotReady) __builtin_ia32_pause();
  if (e != hipSuccess) return fail(c, SGV_ERR_HIP, "metrics wait: %s", hipGetErrorString(e));
  std::memcpy(out4, c->h_met, sizeof(double) * 4);
  c->met_pending = 0;
  return SGV_OK;
}

// ---------------------------------------------------------------------------
// operator seam (tests): R_s v and a batched CG on (c1 R_s + c2 I)
// ---------------------------------------------------------------------------
extern "C" int sgv_ld_matvec(sgv_ctx* c, int ld, int ncol, const double* v, double* y) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || ncol < 1 || ncol > MAXC || !v || !y)
    return fail(c, SGV_ERR_ARG, "sgv_ld_matvec: bad arguments");
  PassArgs pa{};
  for (int j = 0; j < ncol; ++j) {
    CHK(upload_vec(c, v + (size_t)j * c->Mloc, c->S[j]));
    pa.in[j] = c->S[j];
    pa.out[j] = c->S[MAXC + j];
    pa.dot[j] = nullptr;
    pa.c1[j] = 1.0 - c->s;
    pa.c2[j] = c->s;
  }
  CHK(ld_pass(c, ld, ncol, pa));
  for (int j = 0; j < ncol; ++j) CHK(download_vec(c, c->S[MAXC + j], y + (size_t)j * c->Mloc));
  resolve_timers(c);
  return SGV_OK;
}

extern "C" int sgv_cg_solve(sgv_ctx* c, int ld, int ncol, const double* c1, const double* c2,
                            const double* b, double* x, int maxiter, double rtol, int* iters_out,
                            int* info_out) {
  ENTER(c);
  if (ld < 0 || ld >= c->nld || ncol < 1 || ncol > MAXC || !c1 || !c2 || !b || !x ||
      !iters_out || !info_out || maxiter < 0)
    return fail(c, SGV_ERR_ARG, "sgv_cg_solve: bad arguments");
  double* SB[MAXC];
  CgCols cc;
  cc.ncol = ncol;
  int warm[MAXC];
  for (int j = 0; j < ncol; ++j) {
    SB[j] = c->S[j];
    cc.X[j] = c->S[MAXC + j];
    cc.Rr[j] = c->S[2 * MAXC + j];
    cc.P[j] = c->S[3 * MAXC + j];
    cc.Q[j] = c->S[4 * MAXC + j];
    cc.col_ld[j] = ld;
    cc.c1[j] = c1[j] * (1.0 - c->s);
    cc.c2[j] = c1[j] * c->s + c2[j];
    CHK(upload_vec(c, b + (size_t)j * c->Mloc, SB[j]));
    CHK(upload_vec(c, x + (size_t)j * c->Mloc, cc.X[j]));
    warm[j] = host_any(x + (size_t)j * c->Mloc, c->Mloc);
  }
  // r = b - A x0 if x0.any() else b (iterative.py:392)
  PassArgs pa{};
  int nc = 0;
  AxpbyArgs ax{};
  for (int j = 0; j < ncol; ++j) {
    HIPCHK(hipMemcpyAsync(cc.Rr[j], SB[j], sizeof(double) * c->Mpad, hipMemcpyDeviceToDevice, c->st));
    ax.y[j] = cc.Rr[j];
    ax.x[j] = cc.Q[j];
    ax.a[j] = 1.0;
    ax.b[j] = warm[j] ? -1.0 : 0.0;
    if (!warm[j]) continue;
    pa.in[nc] = cc.X[j];
    pa.out[nc] = cc.Q[j];
    pa.dot[nc] = nullptr;
    pa.c1[nc] = cc.c1[j];
    pa.c2[nc] = cc.c2[j];
    ++nc;
  }
  ax.ncol = ncol;
  if (nc) CHK(ld_pass(c, ld, nc, pa));
  // map back: the pass wrote Q for warm columns in order; non-warm Q unused (b = 0 weight)
  HIPCHK(launch_axpby(c->d_ch, c->nch, ax, c->st));
  DotsArgs da{};
  da.ncol = 2 * ncol;
  for (int j = 0; j < ncol; ++j) {
    da.x[j] = SB[j];
    da.y[j] = SB[j];
    da.x[ncol + j] = cc.Rr[j];
    da.y[ncol + j] = cc.Rr[j];
    HIPCHK(hipMemcpyAsync(cc.P[j], cc.Rr[j], sizeof(double) * c->Mpad, hipMemcpyDeviceToDevice,
                          c->st));
  }
  if (2 * ncol > MAXC) return fail(c, SGV_ERR_ARG, "sgv_cg_solve: ncol <= %d", MAXC / 2);
  HIPCHK(launch_dots(c->d_ch, c->nch, da, c->d_part, c->st));
  double tot[MAXC];
  CHK(reduce_host(c, MAXC, c->d_ch_begin, tot));
  double rho[MAXC], atol[MAXC];
  int active[MAXC];
  for (int j = 0; j < ncol; ++j) {
    const double bn = std::sqrt(tot[j]);
    atol[j] = std::max(0.0, rtol * bn);
    rho[j] = tot[ncol + j];
    active[j] = 1;
    if (bn == 0.0) {
      HIPCHK(hipMemcpyAsync(cc.X[j], SB[j], sizeof(double) * c->Mpad, hipMemcpyDeviceToDevice, c->st));
      active[j] = 0;
    }
  }
  CHK(cg_run(c, cc, rho, atol, maxiter, active, iters_out, info_out, nullptr));
  for (int j = 0; j < ncol; ++j) CHK(download_vec(c, cc.X[j], x + (size_t)j * c->Mloc));
  return SGV_OK;
}

extern "C" int sgv_timers(sgv_ctx* c, double* t6, int reset) {
  ENTER(c);
  CHK(stream_wait(c));
  resolve_timers(c);
  if (t6) {
    t6[0] = c->ld_ms;
    t6[1] = c->ld_launches;
    t6[2] = c->ld_bytes;
    t6[3] = c->rhs_bytes;
    t6[4] = c->dense_bytes;
    t6[5] = c->aux_bytes;
  }
  if (reset) {
    c->ld_ms = c->ld_launches = c->rhs_bytes = c->ld_bytes = c->dense_bytes = c->aux_bytes = 0.0;
  }
  return SGV_OK;
}

extern "C" int sgv_exchange_stats(sgv_ctx* c, double* out, int reset) {
  ENTER(c);
  if (!out) return fail(c, SGV_ERR_ARG, "sgv_exchange_stats: out is null");
  CHK(stream_wait(c));
  resolve_timers(c);
  const bool cm = c->comm || c->host_ag;
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
  if (reset) {
    c->xchg_n = c->xchg_ms = c->xchg_bytes = 0.0;
    c->em_loops_rep = c->em_loops_ps = 0.0;
    c->host_wait_ms = 0.0;
  }
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

// ---------------------------------------------------------------------------
// one outer iteration in the shim (src/sgvamp.py:222-387 minus the files and
// logs): the host returns to the caller once, not between the phases
// ---------------------------------------------------------------------------
static int step_impl(sgv_ctx* c, int it, int flags, int em_maxit, int nslab,
                     const double* sigmas, const double* a, double* lam_io, double* omegas_io,
                     const double* gam1s, double rho, const double* gamw,
                     const double* alpha1_prev, const double* alpha2_prev,
                     const int8_t* probes, int cg_maxit, double rtol, int out_slot,
                     double* res, int* ires, double* out, int* cg_out, int staged) {
  if (!sigmas || !a || !lam_io || !omegas_io || !gam1s || !gamw || !alpha1_prev ||
      !alpha2_prev || !probes || !res || !ires || !out || !cg_out || out_slot >= NOUT_SLOTS)
    return fail(c, SGV_ERR_ARG, "sgv_step: bad arguments");
  const int K = c->K;
  c->chain.valid = 0;   // a step chained behind this one fails unless this one completes
  res[0] = 0.0;
  ires[0] = 0;
  // this step's probes go up now, behind nothing: the copy overlaps EM/denoiser
  // (a step begun behind another had its host copy made by sgv_step_begin)
  if (staged >= 0) CHK(probe_issue(c, staged, &c->pref_slot));
  else CHK(probe_upload(c, probes, &c->pref_slot));
  c->pref_src = probes;
  if (flags & SGV_STEP_EM) {   // :250-257
    CHK(sgv_em(c, gam1s, a, nslab, sigmas, em_maxit, lam_io, omegas_io, &ires[0], &res[0]));
  } else if (flags & SGV_STEP_MLE) {   // :244-247
    CHK(sgv_mle_update(c, gam1s, a, nslab, sigmas, lam_io, omegas_io, &c->mle_gam, &ires[0]));
    res[0] = c->mle_gam;
  }
  if (nslab < 1 || nslab > MAXL) return fail(c, SGV_ERR_ARG, "sgv_step: nslab=%d", nslab);
  // denoiser (:270-291); the output copies and metrics (:281-283, 379-387) are
  // queued behind it before the host waits for the derivative sums
  bool met_fused = false;
  CHK(denoise_enqueue(c, gam1s, a, *lam_io, nslab, omegas_io, sigmas, rho,
                      (flags & SGV_STEP_DENOISE_DAMP) ? 1 : 0, (flags & SGV_STEP_METRICS) != 0,
                      &met_fused));
  HIPCHK(hipEventRecord(c->ev_den, c->st));
  if (out_slot >= 0) CHK(sgv_outputs_begin(c, out_slot));
  if ((flags & SGV_STEP_METRICS) && !met_fused) CHK(sgv_metrics_begin(c));
  CHK(event_spin(c, c->ev_den));
  std::vector<double> der(c->h_tot, c->h_tot + K), alpha1(K), gam2(K);
  if (met_fused)   // the metrics' ordered sums (sgv_metrics order), long done
    for (int j = 0; j < 4; ++j) res[1 + 2 * K + j] = c->h_tot[K + j];
  for (int k = 0; k < K; ++k) {
    double a1 = der[k] / (double)c->Mtot;                           // np.mean (:285)
    if (flags & SGV_STEP_ALPHA1_DAMP) a1 = rho * a1 + (1 - rho) * alpha1_prev[k];   // :290-291
    alpha1[k] = a1;
    gam2[k] = gam1s[k] * (1 - a1) / a1;                             // :305
    res[1 + k] = a1;
    res[1 + K + k] = gam2[k];
  }
  int passes = 0;
  CHK(sgv_lmmse(c, it, gamw, gam2.data(), alpha1.data(), alpha2_prev, probes, cg_maxit, rtol,
                (flags & SGV_STEP_LMMSE_DAMP) ? 1 : 0, rho, (flags & SGV_STEP_LEARN_GAMW) ? 1 : 0,
                out, cg_out, &passes));
  ires[1] = passes;
  if ((flags & SGV_STEP_METRICS) && !met_fused) CHK(sgv_metrics_end(c, res + 1 + 2 * K));
  // inputs of a chained next step: src/sgvamp.py:347, 363-374 (gamw clamped to
  // >= 1 after it is logged, as Python's max(gamw, 1.0))
  sgv_ctx::Chain& ch = c->chain;
  for (int k = 0; k < K; ++k) {
    const double* o = out + (size_t)k * SGV_LMMSE_NOUT;
    ch.gam1[k] = o[SGV_O_GAM1];
    const double gw = (flags & SGV_STEP_LEARN_GAMW) ? o[SGV_O_GAMW] : gamw[k];
    ch.gamw[k] = (1.0 > gw) ? 1.0 : gw;
    ch.alpha1[k] = alpha1[k];
    ch.alpha2[k] = o[SGV_O_ALPHA2];
  }
  ch.lam = *lam_io;
  for (int l = 0; l < nslab; ++l) ch.om[l] = omegas_io[l];
  ch.valid = 1;
  return SGV_OK;
}

extern "C" int sgv_step(sgv_ctx* c, int it, int flags, int em_maxit, int nslab,
                        const double* sigmas, const double* a, double* lam_io, double* omegas_io,
                        const double* gam1s, double rho, const double* gamw,
                        const double* alpha1_prev, const double* alpha2_prev,
                        const int8_t* probes, int cg_maxit, double rtol, int out_slot,
                        double* res, int* ires, double* out, int* cg_out) {
  ENTER(c);
  return step_impl(c, it, flags, em_maxit, nslab, sigmas, a, lam_io, omegas_io, gam1s, rho, gamw,
                   alpha1_prev, alpha2_prev, probes, cg_maxit, rtol, out_slot, res, ires, out,
                   cg_out, -1);
}

// Hand-offs spin (a futex wake costs tens of microseconds, the GPU idles for
// it): the worker spins up to ~2 ms for the next step before it blocks, and
// sgv_step_end spins for the step it waits on.  Steps run in begin order.
static void worker_main(sgv_ctx* c) {
  (void)hipSetDevice(c->dev);
  for (;;) {
    sgv_ctx::Job& j = c->jobs[c->job_run % 2];
    const auto t0 = std::chrono::steady_clock::now();
    while (j.state.load(std::memory_order_acquire) != 1 && !c->worker_quit.load()) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
        std::unique_lock<std::mutex> lk(c->wmu);
        c->wcv.wait(lk, [&] { return j.state.load() == 1 || c->worker_quit.load(); });
      }
    }
    if (j.state.load(std::memory_order_acquire) != 1) return;   // quit
    j.state.store(2);
    j.rc = j.fn();
    ++c->job_run;
    j.state.store(3, std::memory_order_release);
  }
}

extern "C" int sgv_step_begin(sgv_ctx* c, int it, int flags, int em_maxit, int nslab,
                              const double* sigmas, const double* a, double* lam_io,
                              double* omegas_io, const double* gam1s, double rho,
                              const double* gamw, const double* alpha1_prev,
                              const double* alpha2_prev, const int8_t* probes, int cg_maxit,
                              double rtol, int out_slot, double* res, int* ires, double* out,
                              int* cg_out) {
  if (!c) return fail(nullptr, SGV_ERR_ARG, "null context");
  if (nslab < 1 || nslab > MAXL || !sigmas || !a || !gam1s || !gamw || !alpha1_prev ||
      !alpha2_prev || !lam_io || !omegas_io)
    return fail(c, SGV_ERR_ARG, "sgv_step_begin: bad arguments");
  sgv_ctx::Job& j = c->jobs[c->job_begun % 2];
  if (j.state.load() != 0) return fail(c, SGV_ERR_ARG, "sgv_step_begin: two steps already queued");
  // the K- and L-length inputs are copied (a chained step takes gam1, gamw,
  // alpha1, alpha2, lam and omegas from the step before it when it starts);
  // lam_io/omegas_io, probes and the outputs stay the caller's until sgv_step_end
  const int K = c->K;
  std::vector<double> v_sig(sigmas, sigmas + nslab), v_a(a, a + K), v_g1(gam1s, gam1s + K),
      v_gw(gamw, gamw + K), v_a1(alpha1_prev, alpha1_prev + K), v_a2(alpha2_prev, alpha2_prev + K);
  // the probes' host copy is made here, while the step ahead runs on the GPU,
  // so the worker starts this step with the device copy alone (the buffers
  // come from the first step's upload; until then the worker stages them)
  int staged = -1;
  if (probes && c->probe_cap.load(std::memory_order_acquire) >= std::max<size_t>((size_t)K * c->Mloc, 8)) {
    staged = probe_stage(c, probes);
    if (staged < 0) return SGV_ERR_HIP;
  }
  j.fn = [=]() mutable {
    if (flags & SGV_STEP_CHAIN) {
      const sgv_ctx::Chain& ch = c->chain;
      if (!ch.valid) return fail(c, SGV_ERR_ARG, "chained step without a completed step");
      for (int k = 0; k < K; ++k) {
        v_g1[k] = ch.gam1[k];
        v_gw[k] = ch.gamw[k];
        v_a1[k] = ch.alpha1[k];
        v_a2[k] = ch.alpha2[k];
      }
      *lam_io = ch.lam;
      for (int l = 0; l < nslab; ++l) omegas_io[l] = ch.om[l];
    }
    ENTER(c);
    return step_impl(c, it, flags & ~SGV_STEP_CHAIN, em_maxit, nslab, v_sig.data(), v_a.data(),
                     lam_io, omegas_io, v_g1.data(), rho, v_gw.data(), v_a1.data(), v_a2.data(),
                     probes, cg_maxit, rtol, out_slot, res, ires, out, cg_out, staged);
  };
  {
    std::lock_guard<std::mutex> lk(c->wmu);   // a worker about to block sees the job
    j.state.store(1, std::memory_order_release);
  }
  ++c->job_begun;
  if (!c->worker.joinable()) c->worker = std::thread(worker_main, c);
  c->wcv.notify_all();
  return SGV_OK;
}

extern "C" int sgv_step_end(sgv_ctx* c) {
  if (!c) return fail(nullptr, SGV_ERR_ARG, "null context");
  if (c->job_ended == c->job_begun) return fail(c, SGV_ERR_ARG, "sgv_step_end without sgv_step_begin");
  sgv_ctx::Job& j = c->jobs[c->job_ended % 2];
  while (j.state.load(std::memory_order_acquire) != 3) __builtin_ia32_pause();
  const int rc = j.rc;
  j.fn = nullptr;
  j.state.store(0);
  ++c->job_ended;
  return rc;
}
