// Internal declarations of the host side of libsgvamp_hip.so: the context
// (sgv_ctx: device buffers, streams, communicator, solver state), the LD
// storage and launch-plan records, the error macros, and the helpers the host
// units share.  The units: capi.hip (lifetime, staging, vectors, generator,
// timers), exchange.hip (the ordered cross-rank reductions, RCCL / host
// exchange, the EM exchange model), ldplan.hip (LD storage, pass plans, the LD
// pass), solver.hip (CG, LMMSE, denoiser, EM, MLE, the step driver).
#pragma once
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
  // band walks (band_walk.hip, 3-8 columns): when every packed block is a band
  // of extent <= WALK_RMAX panels; the walk panel / item tables in creation
  // order, the head panels' finalize table, head / carry slot counts
  SymWalk* d_walks = nullptr;
  int nwalks = 0;
  SymPanel* d_wpanels = nullptr;
  SymItem* d_witems = nullptr;
  WalkFin* d_wfins = nullptr;
  int nwfins = 0, nhslots = 0, ncslots = 0;
  double stored_bytes = 0.0, dense_bytes = 0.0;
  // multiply-adds per column of a pass: every stored element (row part) plus the
  // packed off-diagonal-block ones again (their transposes)
  double mac_elems = 0.0;
  // coupled band pieces: k_coupling_lds tasks, panel slots of PassArgs::cpbuf, and
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

// chunk-width class of the packed VALU pass for nc columns (CW = 1024 >> cls)
static inline int sym_class(int nc) { return nc <= 2 ? 0 : nc <= 4 ? 1 : nc <= 8 ? 2 : 3; }
// default number of right-hand sides from which packed passes run on the f64
// matrix cores (sym_mfma.hip, class-1 items); per context: sgv_set_mfma_min
// (0 disables)
static inline int mfma_min_default() { return 3; }
// CG loop driver: 1 (default) = pipelined, device-side control (cg_loop_dev);
// 0 = host-side stop test per iteration (cg_loop).  Env SGV_CG_PIPE.
static inline int cg_pipe_default() {
  const char* e = ab_env("SGV_CG_PIPE");
  return (e && e[0] == '0') ? 0 : 1;
}
constexpr int CG_RING = 4;   // mirror slots of the pipelined CG
constexpr int MAXGRP = 8;    // block groups of one MFMA pass (pass_groups)
constexpr int NOUT_SLOTS = 3;   // pinned output slots (a writer reads one while two steps run)

// SGV_CG_EXACT=0: the pipelined CG's pass of iteration it also carries the
// columns that stop at it's own test (one iteration of look-ahead; A/B);
// sgv_set_cg_exact sets the run's mode (the Engine: from the global LD size)
static inline int cg_exact_default() {   // -1: by size (cg_loop_dev); 0 / 1 forced (A/B)
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
static inline int sym_class_nc(int cls) { return std::min(16, 2 << (cls + 1)); }   // widest NC using cls

// The one-workgroup reduction + control kernels (k_cg_reduce_ctl,
// k_em_reduce_ctl) walk nv x nblk (value, block) pairs 128 at a time, each round
// a chain of dependent loads; above one round the two-launch form (k_reduce_local
// over nv workgroups, then the one-wave control kernel; the same bits) is
// faster: at 64 blocks 58 / 40 us fused vs ~9 + 5 us (north-star trace).
static inline bool fused_ctl_pays(int nv, int nblk) {
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
  double* d_whead = nullptr;     // band walks: head panels' partial sums [slot][256][8]
  double* d_wcarry = nullptr;    // band walks: open ring slots at a walk's end [slot][256][8]
  size_t whead_cap = 0, wcarry_cap = 0;
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
  // exact CG column sets: the device's idle time between the p update and the
  // passes the host enqueues once it has read the stop test (HIP events)
  double host_wait_ms = 0.0;
  // device-loop EM prior loops timed with HIP events (first enqueue to the
  // last step's completion), to check the cost model against
  double em_ms = 0.0, em_loops_timed = 0.0;
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
  std::vector<int> pending_wide;   // the pass ran 9..16 columns (16x16x4 MFMA)
  // cross-rank exchange counters (sgv_exchange_stats): all-gathers issued, the
  // bytes each rank contributed, and their time -- HIP events around every
  // ncclAllGather on the ctx stream (the wait for the slowest peer included),
  // wall time of the host callback for the host exchange
  std::vector<std::pair<hipEvent_t, hipEvent_t>> xpending;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> gpending;   // exact-CG read gaps
  std::vector<std::pair<hipEvent_t, hipEvent_t>> empending;  // EM loops
  double xchg_n = 0.0, xchg_ms = 0.0, xchg_bytes = 0.0;
  double ld_ms = 0.0, ld_launches = 0.0, rhs_bytes = 0.0, ld_bytes = 0.0, dense_bytes = 0.0,
         aux_bytes = 0.0;
  // algorithmic flops of the passes (2 per multiply-add: row part of every stored
  // element, column part of the packed off-diagonal-block ones), and the 9..16-
  // column passes' share (their bound is the f64 matrix core, not HBM)
  double ld_flops = 0.0, ld_flops_wide = 0.0, ld_ms_wide = 0.0, ld_launches_wide = 0.0;
  std::string err;
};

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

static inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------
static inline Map16 identity_map() {
  Map16 m;
  for (int i = 0; i < MAXNV; ++i) m.d[i] = i;
  return m;
}


// ---------------------------------------------------------------------------
// helpers shared by the host units (defined where noted)
// ---------------------------------------------------------------------------
// capi.hip
int fail(sgv_ctx* c, int code, const char* fmt, ...);
int stream_wait(sgv_ctx* c);
void resolve_timers(sgv_ctx* c);
int event_pair(sgv_ctx* c, hipEvent_t* e0, hipEvent_t* e1);
int ensure_stage(sgv_ctx* c, size_t bytes);
int ensure_hstage(sgv_ctx* c, size_t bytes);
int probe_stage(sgv_ctx* c, const int8_t* probes);
int probe_upload(sgv_ctx* c, const int8_t* probes, int* slot_out);
int probe_issue(sgv_ctx* c, int slot, int* slot_out);
int upload_vec(sgv_ctx* c, const double* host, double* dpad);
int download_vec(sgv_ctx* c, const double* dpad, double* host);
bool host_any(const double* v, int64_t n);
// exchange.hip
int reduce_dev(sgv_ctx* c, int nv, const int* d_begin, const Map16& map, double* d_dst,
               int op = 0);
int reduce_dev2(sgv_ctx* c, const double* partA, int nvA, const int* beginA, int nvB,
                const int* beginB, const Map16& mapB, int offB, double* d_dst);
int reduce_host(sgv_ctx* c, int nv, const int* d_begin, double* out, int op = 0);
int gather_f64(sgv_ctx* c, const double* d_send, double* d_recv, size_t cnt, double* h_send,
               double* h_recv);
bool em_mode_pick(sgv_ctx* c, int maxit);
int gather_r1(sgv_ctx* c);
// ldplan.hip
void free_plan(LdPlan& p);
void free_block(LdBlock& lb);
int ld_alloc(sgv_ctx* c, int ld, int b, int fmt, int64_t ext = 0);
int grow(sgv_ctx* c, double** buf, size_t* cap, size_t need);
int ensure_plan(sgv_ctx* c, int ld);
const int* ld_parts(sgv_ctx* c, int ld);
int ld_pass(sgv_ctx* c, int ld, int nc, const PassArgs& pa_in);

// a host table -> a new device array (*d; nothing for an empty table)
template <typename T>
static inline int upload_table(sgv_ctx* c, const std::vector<T>& h, T** d) {
  if (h.empty()) return SGV_OK;
  HIPCHK(hipMalloc(d, sizeof(T) * h.size()));
  HIPCHK(hipMemcpy(*d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  return SGV_OK;
}
