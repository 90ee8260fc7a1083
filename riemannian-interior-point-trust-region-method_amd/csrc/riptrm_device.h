// riptrm_device.h — device-side layout shared by the kernels and the C-ABI host code.
//
// Workspace (one allocation, caller-owned, zeroed at bind):
//   [vectors]  NVEC x batch x ld doubles          per-instance state vectors (SoA per kind)
//   [state]    batch x ST_N doubles               per-instance scalars (see enum St)
//   [stats]    batch x RIPTRM_STAT_NFIELDS        host-visible results
//   [log]      batch x cap x RIPTRM_LOG_NFIELDS   per-inner-iteration log rows
//   [pbuf]     2 x batch x nt x nt x TS doubles   S-pass partial sums (symmetric-tile layout)
//              MM_KZ x 2 x batch x ld doubles    K-slice partial products (shared layout)
//   [lists]    4 x batch int32                    active-instance lists (2 groups x ping-pong)
//   [req]      batch int32                        right-hand sides wanted per instance (1|2)
//   [counters] 4 int32                            list lengths (2 groups x ping-pong)
#pragma once
#include <stdint.h>
#include "../../include/riptrm.h"

namespace riptrm {

// S layouts (RIPTRM_LAYOUT_*): full row-major, or the upper triangle in TS x TS tiles
constexpr int TS = 128;            // tile edge of the symmetric-tile layout; vector padding unit
constexpr int SP_WAVES = 8;        // waves per tile workgroup, 16 rows each
constexpr int SP_THREADS = SP_WAVES * 64;
// rows of S handled by one full-layout mat-vec workgroup (4 waves x GV_RW rows)
constexpr int GV_THREADS = 256;
constexpr int GV_RW = 4;
constexpr int GV_RB = (GV_THREADS / 64) * GV_RW;
// state-machine workgroup
constexpr int ST_THREADS = 512;
constexpr int ST_WAVES = ST_THREADS / 64;

// state vector kinds
enum Vec : int {
  V_X = 0, V_Y, V_ETA, V_HETA,   // 0..3 fixed so riptrm_workspace_offset kinds 0..3 map here
  V_SX, V_X0, V_Y0, V_SX0, V_XPREV, V_R, V_IN0, V_IN1, V_OUT0, V_OUT1, V_YNEW, V_C,
  V_XI, V_YI, V_SXI,             // initial point (restart_every cycling)
  NVEC
};

// per-instance scalar slots (all stored as double; integers are exact below 2^53)
enum St : int {
  ST_PHASE = 0, ST_MODE, ST_OUTER_IT, ST_INNER_IT, ST_MU_IDX, ST_MU, ST_DELTA, ST_DELTA0,
  ST_DELTA_STEP, ST_T_START, ST_T_INNER, ST_TOLL, ST_TOLC,
  // hoisted per inner step
  ST_XX, ST_XSX, ST_YX, ST_COEF, ST_FCUR,
  // tCG
  ST_EPE, ST_EPD, ST_DPD, ST_ZR, ST_NORMR0, ST_MODEL, ST_J, ST_TCG_STOP,
  // trial
  ST_NORMDX, ST_XDX, ST_MINX, ST_MINY, ST_COMPL, ST_XFEAS, ST_YFEAS,
  // Exact_RepMat second-order test at the trial point (RIPTRM.py:599-613)
  ST_HASMIN, ST_MINEIG, ST_MINEIG_OK,
  ST_HOT_END,
  // cold: thread-0-owned counters
  ST_TCG_TOTAL = 40, ST_INNER_TOTAL, ST_PASSES, ST_LOG_COUNT, ST_LOG_OVERFLOW, ST_STOP_CODE,
  ST_STOP_RUNTIME, ST_RESIDUAL,
  // last inner_info (for save_inner_iteration == False rows)
  ST_I_HAS, ST_I_NUM, ST_I_STATUS, ST_I_TR, ST_I_DXTYPE, ST_I_NORMDX, ST_I_MINX, ST_I_MINY,
  ST_I_COMPL, ST_I_HASRATIO, ST_I_RATIO, ST_I_RU, ST_I_DC, ST_I_HASMIN, ST_I_MINEIG,
  ST_ERROR, ST_LOG_BASE, ST_RHS,
  ST_N_USED
};
constexpr int ST_N = 72;
constexpr int ST_HOT = ST_HOT_END;
static_assert(ST_HOT_END <= 40, "hot scalar slots overflow into cold ones");
static_assert(ST_N_USED <= ST_N, "state slots overflow");

enum Phase : int {
  PH_IDLE = 0, PH_START, PH_AFTER_SX0, PH_TCG, PH_TRIAL, PH_PAUSED, PH_DONE,
  PH_TCGO_START, PH_TCGO_SX, PH_ERROR,
  PH_TRS, PH_TRS_END,  // Exact_RepMat: subproblem solve / rest of the inner step (no S-pass between)
  // Exact_RepMat above RIPTRM_TRS_DIM_MAX (riptrm_trs_big.hip): parked until the host has served the
  // subproblem (-> PH_TRS_END) or the trial point's smallest eigenvalue (-> PH_MINEIG_END)
  PH_TRS_HOST, PH_MINEIG_HOST, PH_MINEIG_END
};

enum Mode : int { MODE_SOLVE = 0, MODE_TCG_ONLY = 1 };

struct Layout {
  int32_t n, batch, cap, layout, nt;
  int32_t reps;        // persistent-mode replicas per instance (0: the layout has no persistent region)
  int64_t ld;
  int64_t off_vec, off_state, off_stats, off_log, off_pbuf, off_lists, off_req, off_cnt;
  // persistent mode (k_persist): the replicas' private state (vectors, scalars, stats, requests)
  // for batch x (reps - 1) replicas, the second parity of the partial grid, and the sync block
  // (per-instance arrival counters + published clocks + the timeout flag; zeroed before every launch)
  int64_t off_rvec, off_rstate, off_rstats, off_rreq, off_pbuf2, off_sync, sync_bytes, off_tgrid, tgrid_bytes;
  int64_t total;
};

inline int64_t round_up(int64_t a, int64_t m) { return (a + m - 1) / m * m; }

// log slot of record k (counted from the last rebase) in a log of `cap` slots: linear while
// k < cap, then the first cap/2 slots keep the head and the rest is a ring of the latest records
// (include/riptrm.h "Log slots").  cap >= 1.
__host__ __device__ inline int64_t log_slot(int64_t k, int64_t cap) {
  if (k < cap) return k;
  const int64_t h = cap / 2, t = cap - h;
  return h + (k - h) % t;
}
inline int64_t ld_of(int32_t n) { return round_up(n > 0 ? n : 1, TS); }
inline int64_t rows_of(int32_t n) { return round_up(n > 0 ? n : 1, 32); }  // k_pack writes 32-row sub-tiles
inline int32_t nt_of(int32_t n) { return (int32_t)(ld_of(n) / TS); }
inline int64_t ntiles_of(int32_t n) { const int64_t t = nt_of(n); return t * (t + 1) / 2; }
// Persistent super-tile S-pass (k_spass_sup): work units of SB x SB stored tiles, partial sums
// of SW = SB TS elements per unit side; nst super-blocks per dimension
constexpr int SB = 2;
constexpr int SW = SB * TS;
inline int32_t nst_of(int32_t n) { return (nt_of(n) + SB - 1) / SB; }
inline int64_t nsup_of(int32_t n) { const int64_t t = nst_of(n); return t * (t + 1) / 2; }
// doubles of one instance's S-pass partial grid (one right-hand side): the larger of the tile
// grid [nt][nt][TS] and the super-tile grid [nst][nst][SW]
inline int64_t pgrid_of(int32_t n) {
  const int64_t a = (int64_t)nt_of(n) * nt_of(n) * TS, b = (int64_t)nst_of(n) * nst_of(n) * SW;
  return a > b ? a : b;
}
// shared-S MFMA S-pass: K is split over MM_KZ workgroup slices whose partial products land in
// MM_KZ x 2 x batch x ld slabs, summed in slice order by the state kernel
#ifndef RIPTRM_MM_KZ
#define RIPTRM_MM_KZ 4   // A/B builds: -DRIPTRM_MM_KZ=8 (scripts/gpu_r3mm.sh)
#endif
constexpr int MM_KZ = RIPTRM_MM_KZ;  // csrc/riptrm_kernels.hip k_spass_mm: 4 vs 8 slices measured

// Symmetric-tile layout: tiles (I, J), I <= J, row by row; full TS x TS tiles except the last
// tile column (J = nt - 1), which keeps only the wl = round_up(n - (nt - 1) TS, 32) columns that
// hold data (row stride wl), and the corner tile (nt - 1, nt - 1), wl x wl.  wl = TS when n is a
// multiple of TS.  Offset of tile (I, J) = base(I) + (J - I) TS^2.
inline int32_t edge_w_of(int32_t n) {
  return (int32_t)round_up((int64_t)(n > 0 ? n : 1) - (int64_t)(nt_of(n) - 1) * TS, 32);
}
__host__ __device__ inline int64_t sym_off(int I, int J, int nt, int wl) {
  const int64_t F = (int64_t)TS * TS;
  return F * ((int64_t)I * (nt - 1) - (int64_t)I * (I - 1) / 2) + (int64_t)I * TS * wl + (int64_t)(J - I) * F;
}

// doubles of one instance of S in a layout
inline int64_t s_elems_of(int32_t n, int32_t layout) {
  if (layout == RIPTRM_LAYOUT_SYMTILE) {
    const int nt = nt_of(n), wl = edge_w_of(n);
    return sym_off(nt - 1, nt - 1, nt, wl) + (int64_t)wl * wl;
  }
  return rows_of(n) * ld_of(n);
}

// Persistent lock-step mode (k_persist; symmetric-tile layout, tCG): one 512-thread workgroup per
// stored tile of every instance, all co-resident (one per CU: the tile sits in 128 KiB of LDS), so
// at most PERSIST_MAX_WG workgroups; every workgroup of an instance runs a private replica of the
// instance's state machine.  The workspace carries the replica region whenever the shape allows it;
// riptrm_nonnegpca_bind enables the mode only if the device has that many CUs.
constexpr int PERSIST_MAX_WG = 256;
constexpr int PERSIST_MAX_N = 2048;   // nt <= 16: 136 tiles
inline int32_t persist_reps_of(int32_t n, int32_t batch, int32_t layout) {
  if (layout != RIPTRM_LAYOUT_SYMTILE || n > PERSIST_MAX_N) return 0;
  const int64_t t = ntiles_of(n);
  return (int64_t)batch * t <= PERSIST_MAX_WG ? (int32_t)t : 0;
}

inline Layout make_layout(int32_t n, int32_t batch, int32_t cap, int32_t layout) {
  Layout L;
  L.n = n; L.batch = batch; L.cap = cap; L.ld = ld_of(n); L.layout = layout; L.nt = nt_of(n);
  int64_t o = 0;
  L.off_vec = o;   o += (int64_t)NVEC * batch * L.ld * 8;               o = round_up(o, 256);
  L.off_state = o; o += (int64_t)batch * ST_N * 8;                       o = round_up(o, 256);
  L.off_stats = o; o += (int64_t)batch * RIPTRM_STAT_NFIELDS * 8;        o = round_up(o, 256);
  L.off_log = o;   o += (int64_t)batch * cap * RIPTRM_LOG_NFIELDS * 8;   o = round_up(o, 256);
  L.off_pbuf = o;
  if (layout == RIPTRM_LAYOUT_SYMTILE) o += (int64_t)2 * batch * pgrid_of(n) * 8;
  if (layout == RIPTRM_LAYOUT_SHARED) o += (int64_t)MM_KZ * 2 * batch * L.ld * 8;
  o = round_up(o, 256);
  L.off_lists = o; o += (int64_t)4 * batch * 4;                          o = round_up(o, 256);
  L.off_req = o;   o += (int64_t)batch * 4;                              o = round_up(o, 256);
  L.off_cnt = o;   o += 64;   // [0..3] list counts, [8..11] S-pass unit tickets, [12..15] done counts                                              o = round_up(o, 256);
  L.reps = persist_reps_of(n, batch, layout);
  const int64_t bs = L.reps > 0 ? (int64_t)batch * (L.reps - 1) : 0;   // replicas beyond the instance itself
  L.off_rvec = o;   o += (int64_t)NVEC * bs * L.ld * 8;                  o = round_up(o, 256);
  L.off_rstate = o; o += bs * ST_N * 8;                                  o = round_up(o, 256);
  L.off_rstats = o; o += bs * RIPTRM_STAT_NFIELDS * 8;                   o = round_up(o, 256);
  L.off_rreq = o;   o += bs * 4;                                         o = round_up(o, 256);
  L.off_pbuf2 = o;  if (L.reps > 0) o += (int64_t)2 * batch * pgrid_of(n) * 8;  o = round_up(o, 256);
  L.off_sync = o;
  L.sync_bytes = L.reps > 0 ? round_up((int64_t)batch * 4, 16) + (int64_t)2 * batch * 8 + 16 : 0;
  o += L.sync_bytes;                                                     o = round_up(o, 256);
  // the tagged grid of lean tCG passes right after the sync block (one memset zeroes both)
  L.off_tgrid = o;
  L.tgrid_bytes = L.reps > 0 ? (int64_t)2 * batch * nt_of(n) * nt_of(n) * TS * 16 : 0;
  o += L.tgrid_bytes;                                                    o = round_up(o, 256);
  L.total = o;
  return L;
}

// Kernel parameter block (passed by value).
struct DevParams {
  const double* S;      // batch instances, inst_stride doubles apart (layout below)
  int64_t inst_stride;  // doubles between instances of S
  int64_t ld;
  int32_t n, batch, cap;
  int32_t nrb;          // row blocks per instance (full layout)
  int32_t layout;       // RIPTRM_LAYOUT_*
  int32_t nt;           // tiles per dimension (symmetric-tile layout)
  int32_t ntiles;       // nt (nt + 1) / 2
  int32_t wl;           // stored columns of the last tile column (symmetric-tile layout)
  int32_t nst, nsup;    // super-blocks per dimension, super-tile units per instance
  int32_t smode;        // per launch: 0 = tile S-pass (grid [nt][nt][TS]), 1 = super-tile ([nst][nst][SW])
  int32_t sup_dyn;      // k_spass_sup: 1 = units handed out by a ticket counter (cnt[8 + list]), 0 = static
  double* pbuf;         // S-pass partial sums: 2 x pbatch x pgrid_of(n) (symmetric-tile layout),
                        // MM_KZ x 2 x batch x ld (shared layout)
  int32_t pbatch;       // instances of the partial grid (= batch; the persistent replicas' parameter
                        // block has batch = replica count but shares the instances' grid)
  double* vec;          // workspace vectors
  double* st;           // workspace scalars
  double* stats;
  double* log;
  int32_t* lists;       // 4 x batch: list id = group * 2 + parity
  int32_t* req;
  int32_t* cnt;
  const double* mu_tab;
  const double* tolL_tab;
  const double* tolC_tab;
  int32_t tab_len;
  int32_t outer_target;
  double clock_hz;
  int32_t trs_hbm;      // 1: Exact_RepMat's subproblems on the HBM path at every n (RIPTRM_TRS_HBM=1; A/B)
  riptrm_options opt;
};

}  // namespace riptrm
