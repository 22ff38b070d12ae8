// LD storage and the LD pass of libsgvamp_hip.so: dense / packed-triangle /
// packed-band blocks (src/main.py:199-202, 251-257, 265), their launch plans
// (MFMA strips in block groups, band walks, couplings between band pieces)
// and ld_pass, the operator of every CG iteration (src/sgvamp.py:312-316, 332;
// A = gamw R_s + gam2 I is never built: the pass's fused epilogue).
#include "ctx.h"

// ---------------------------------------------------------------------------
// LD pass (timed with HIP events on the ctx stream)
// ---------------------------------------------------------------------------
void free_plan(LdPlan& p){
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
  if (p.d_walks) (void)hipFree(p.d_walks);
  if (p.d_wpanels) (void)hipFree(p.d_wpanels);
  if (p.d_witems) (void)hipFree(p.d_witems);
  if (p.d_wfins) (void)hipFree(p.d_wfins);
  p = LdPlan();
}

void free_block(LdBlock& lb){
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
int ld_alloc(sgv_ctx* c, int ld, int b, int fmt, int64_t ext){
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

int grow(sgv_ctx* c, double** buf, size_t* cap, size_t need){
  if (need <= *cap) return SGV_OK;
  if (*buf) HIPCHK(hipFree(*buf));
  *buf = nullptr;
  HIPCHK(hipMalloc(buf, sizeof(double) * need));
  *cap = need;
  return SGV_OK;
}


// panels per MFMA strip (a function of nothing but the block's panels, so the
// sums are the same on every rank count; 3-32 panels and 5-panel strips for
// short launches measured in rounds 1-4, profiles/r04/strip5_ab.jsonl)
constexpr int MFMA_STRIP = 8;

// Block groups of the MFMA pass: one group per ~4 rounds of strips on the
// device's workgroup slots, at most 8 -- a group's finalize then overlaps the
// next group's strips on a second stream.  The grouping changes no sum (strips
// and panels are the same work items in another launch), so products are
// bitwise the same for every count (1, 2, 4, 8 groups: profiles/r05/
// pass_groups_ab.jsonl); it is a function of this rank's plan only.
static int pass_groups(int nstrips, int nblk, int slots) {
  const int g = nstrips / std::max(1, 4 * slots);
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
// choice is free per plan.  Auto (1): the pair kernel for the plan's 3-8-column
// passes when its launch drains with at least 3 % less tail by the strips'
// model cost (a few strips per slot: an 8-block share of the north star, 0.924
// against 0.986 of a perfect split; 16 blocks and 8 x 25,000 stay on the 4-wave
// kernel); SGV_MF_PAIR=0 / 1 (with SGV_AB=1) forces none / every pass (2).
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
  const int S = MFMA_STRIP;
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
  // +4-7 %, the 8-block share -1 %).  Round 6: workgroup i runs on XCD i mod 8
  // (tools/strip_trace.py), and in creation order a chunk's top strips fall
  // 8:4 on the even XCDs, whose busy time ran up to 18 % above the odd ones';
  // dealing each strip kind evenly over the XCDs (by place in its chunk)
  // evened seven of the eight but left the pass even on the 8-block share and
  // +0.8 / +2 % on 64 x 15,625 / 8 x 25,000 (profiles/r06/strip_order_*.jsonl,
  // strip_trace_xcd_*.jsonl): the pass is bound by the HBM side, not by which
  // XCD drains last.
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

// Band walks of LD matrix ld (band_walk.hip) from the class-1 tables in
// creation order, when every packed block is a band whose stored extent is at
// most WALK_RMAX panels (R = extent / 256): each block's panels are cut into
// walks of W = max(4, 2 (R - 1)) -- a function of the block alone, so the
// summation order is the same for every rank count; W >= R - 1 keeps every
// column part inside the walk or the one before it.  A walk that does not start
// its block has min(R - 1, np) head panels; one that does not end it leaves
// min(R - 1, panels after it) carry slots.
// The walks run the band passes of up to 8 columns (two 4x4x4 column groups;
// 9-16 columns stay on the strips' 16x16x4 kernel): at M = 1e6, bw = 1,000
// 1.68 / 1.71 / 1.99 ms at 3 / 4 / 8 columns against the strips' 1.87 / 1.92
// / 2.12 (profiles/r05/walk_ab/wvs_a_ab.jsonl).
// SGV_BAND_WALK=0 (with SGV_AB=1): the strips for every band pass (the
// walks-vs-strips A/B of tools/gpu_walk_vs_strips.sh).
static int band_walk_max_nc() {
  const char* e = ab_env("SGV_BAND_WALK");
  return (e && e[0] == '0') ? 0 : 8;
}

static int plan_walks(sgv_ctx* c, int ld, const std::vector<SymItem>& items,
                      const std::vector<SymPanel>& panels, LdPlan* pl) {
  if (band_walk_max_nc() == 0) return SGV_OK;
  bool any = false;
  for (int b = 0; b < c->nblk; ++b) {
    const LdBlock& lb = c->ldb[ld][b];
    if (lb.fmt != 1) continue;
    if (lb.ext <= 0 || lb.ext > (int64_t)WALK_RMAX * SYM_H) return SGV_OK;
    // the walk kernel addresses a block's Pk rows with 32-bit byte offsets
    // (row * 8 * PKS, PKS <= 8): a block of 2^31 / 64 rows or more takes the
    // strips (~33.5M markers, beyond a chromosome of SNPs)
    if (c->bn[b] + SYM_H >= ((int64_t)1 << 31) / (8 * 8)) return SGV_OK;
    any = true;
  }
  if (!any) return SGV_OK;
  std::vector<SymWalk> walks;
  std::vector<WalkFin> fins;
  int hs = 0, cs = 0, bp0 = 0;
  for (int b = 0; b < c->nblk; ++b) {
    const LdBlock& lb = c->ldb[ld][b];
    if (lb.fmt != 1) continue;
    const int np = (int)lb.poff.size();
    const int R = (int)(lb.ext / SYM_H);
    // walk length 2 (R - 1): measured against 6, 12 and 16 panels at R = 5 (round 6,
    // profiles/r06/walklen_*.jsonl): 6 +12 %, 12 +43 % (1.3 rounds of walks on the 256
    // CUs), 16 even -- the count of walks against the CUs matters more than the
    // head-panel share
    const int W = std::max(4, 2 * (R - 1));
    int prev_cslot = -1;
    for (int g0 = 0; g0 < np; g0 += W) {
      SymWalk w;
      w.p0 = bp0 + g0;
      w.np = std::min(W, np - g0);
      w.nhead = g0 > 0 ? std::min(R - 1, w.np) : 0;
      w.ncarry = std::min(R - 1, np - (g0 + w.np));
      w.hslot = hs;
      w.cslot = cs;
      w.R = R;
      w.pad_ = 0;
      for (int j = 0; j < w.nhead; ++j) fins.push_back(WalkFin{w.p0 + j, hs + j, prev_cslot + j, 0});
      hs += w.nhead;
      prev_cslot = cs;
      cs += w.ncarry;
      walks.push_back(w);
    }
    bp0 += np;
  }
  // longest walks first (a block's last walk can be short); order changes no sum
  std::stable_sort(walks.begin(), walks.end(),
                   [](const SymWalk& a, const SymWalk& b) { return a.np > b.np; });
  pl->nwalks = (int)walks.size();
  pl->nwfins = (int)fins.size();
  pl->nhslots = hs;
  pl->ncslots = cs;
  CHK(upload_table(c, walks, &pl->d_walks));
  CHK(upload_table(c, fins, &pl->d_wfins));
  CHK(upload_table(c, panels, &pl->d_wpanels));
  CHK(upload_table(c, items, &pl->d_witems));
  CHK(grow(c, &c->d_whead, &c->whead_cap, (size_t)std::max(hs, 1) * SYM_H * 8));
  CHK(grow(c, &c->d_wcarry, &c->wcarry_cap, (size_t)std::max(cs, 1) * SYM_H * 8));
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
  // a piece's head rows (coupling gb - 1: nc) and tail rows (coupling gb: nr)
  // must not overlap: both couplings store their sums into the same panel slots
  for (size_t i = 1; i < cv.size(); ++i) {
    if (cv[i].gb != cv[i - 1].gb + 1) continue;
    const int b = cv[i].gb - c->blk0;
    if (b >= 0 && b < c->nblk && (int64_t)cv[i - 1].nc + cv[i].nr > c->bn[b])
      return fail(c, SGV_ERR_ARG,
                  "couplings %d and %d overlap in piece %d: %d head + %d tail rows > %lld markers",
                  cv[i - 1].gb, cv[i].gb, cv[i].gb, cv[i - 1].nc, cv[i].nr, (long long)c->bn[b]);
  }
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
int ensure_plan(sgv_ctx* c, int ld){
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
    pl.mac_elems += lb.stored_bytes / 8.0;
    if (lb.fmt == 1) {   // + the stored elements right of each panel's H x H diagonal block
      double diag = 0.0;
      for (int64_t r0 = 0; r0 < c->bn[b]; r0 += SYM_H) {
        const double H = (double)std::min<int64_t>(SYM_H, c->bn[b] - r0);
        diag += H * H;
      }
      pl.mac_elems += lb.stored_bytes / 8.0 - diag;
    }
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
    if (cls == 1) {
      CHK(build_strips(c, ld, items, panels, &pl));
      CHK(plan_walks(c, ld, items, panels, &pl));
    }
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

const int* ld_parts(sgv_ctx* c, int ld){ return c->plan[ld].d_pbeg; }

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

int ld_pass(sgv_ctx* c, int ld, int nc, const PassArgs& pa_in){
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
      const bool walk = pl.nwalks && nc <= band_walk_max_nc();
      HIPCHK(launch_pk(pa, nc, c->Mpad, c->d_pk, c->st,
                       walk ? nc > 4 : strip_pk_paired(nc)));
      if (walk) {   // band plan: the walks, then the head panels
        HIPCHK(launch_band_walk(nc, pl.d_walks, pl.nwalks, pl.d_wpanels, pl.d_witems, c->d_pk,
                                c->Mpad, pa,
                                c->d_whead, c->d_wcarry, pl.d_wfins, pl.nwfins, c->d_part, c->st));
      } else if (pl.ngrp <= 1) {
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
      if (walk)   // head partials and carries, written and read
        c->aux_bytes += 2.0 * 8.0 * nc * SYM_H * (double)(pl.nhslots + pl.ncslots);
      else
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
  const bool wide = nc > 8 && pl.npanels && c->mfma_min > 0 && nc >= c->mfma_min;
  c->pending_wide.push_back(wide ? 1 : 0);
  c->ld_flops += 2.0 * nc * pl.mac_elems;
  if (wide) {
    c->ld_flops_wide += 2.0 * nc * pl.mac_elems;
    c->ld_launches_wide += 1.0;
  }
  c->ld_launches += 1.0;
  c->ld_bytes += pl.stored_bytes;
  c->dense_bytes += pl.dense_bytes;
  c->rhs_bytes += 2.0 * nc * (double)c->Mloc * 8.0;
  return SGV_OK;
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
