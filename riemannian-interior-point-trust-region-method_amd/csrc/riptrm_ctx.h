// riptrm_ctx.h — host-side context shared by the C-ABI translation units (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include <utility>
#include <vector>
#include "riptrm_device.h"

namespace riptrm_si { struct Bound; }
void riptrm_si_release(riptrm_si::Bound* s);

using riptrm::Layout;
using riptrm::DevParams;

struct riptrm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  bool bound = false, solving = false;
  Layout L{};
  const double* S = nullptr;
  int64_t inst_stride = 0;
  char* ws = nullptr;
  DevParams P{};
  // two instance groups with independent lock-step pipelines on two streams: one group's
  // latency-bound state kernel overlaps the other group's HBM-bound S-pass
  int ngroups = 1;
  int groups_req = 0;  // riptrm_set_stream_groups: 0 = automatic
  int gbase[2] = {0, 0}, gsize[2] = {0, 0};
  int parity[2] = {0, 0};        // list written by the group's last state kernel
  int active_bound[2] = {0, 0};  // upper bound of the group's active instances
  hipStream_t gstream[2] = {nullptr, nullptr};
  hipStream_t own_stream = nullptr;  // created for group 1
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_pass[2] = {nullptr, nullptr};
  double clock_hz = 1e8;
  int ncu = 256;              // compute units (persistent S-pass grid)
  int sup_req = 1;            // riptrm_set_spass_kind: 0 = tile S-pass only, 1 = automatic (fixed rule),
                              // 2 = super-tile always, 3 = automatic with bind-time timing
  int sup_auto = 1;           // kind 3: the super-tile kernel won the bind-time calibration
  float spass_cal_ms[2] = {0.0f, 0.0f};   // calibration: ms per launch of the per-tile / super-tile kernel
  // optional HIP-event timing of every k_gemv / k_state launch (riptrm_profile_*)
  bool prof = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> ev_gemv, ev_state;  // (start, end) indices into ev_pool
  int ev_used = 0;
  double gemv_ms = 0.0, state_ms = 0.0;
  int64_t gemv_n = 0, state_n = 0;
  // hipGraph of GRAPH_STEPS lock-step iterations (single group, no profiling): replayed instead of
  // 2 launches per step when the kernels are short enough for host launch cost to matter
  hipGraphExec_t gexec = nullptr;
  int g_bound = -1, g_parity = -1;
  uint64_t g_pver = ~0ull;
  uint64_t pver = 0;          // bumped whenever P (kernel parameters) changes
  int graphs = 1;             // riptrm_set_graphs
  // persistent lock-step mode (k_persist): requested (riptrm_set_persistent), possible for the
  // bound shape on this device, and active for the current solve (tCG only)
  // persist_req: 0 never, 1 automatic (cooperative launch: co-residency checked by the runtime),
  // 2 automatic with a plain launch (A/B), 3 = 1 with the first launch of each solve treated as
  // refused (tests the lock-step fallback).  persist_launched: a k_persist launch of the current
  // solve has run (after that a refused launch is an error, before it the solve falls back).
  int persist_req = 1;
  bool persist_ok = false, persist_on = false, persist_launched = false;
  int persist_fallbacks = 0;   // solves that fell back to lock-step since bind
  unsigned long long* persist_trace = nullptr;   // riptrm_persist_trace (diagnostics)
  int persist_trace_cap = 0;
  // StableIdentification binding (riptrm_si.hip)
  riptrm_si::Bound* si = nullptr;
  // Exact_RepMat above RIPTRM_TRS_DIM_MAX (riptrm_trs_big.hip): caller-owned scratch bound by
  // riptrm_trs_bind_workspace (slots of order big_order) and the rocBLAS handle of rocSOLVER
  char* big_ws = nullptr;
  int big_order = 0, big_slots = 0;
  void* big_handle = nullptr;
  // per-instance cache of the trial point's eigendecomposition (riptrm_trs_bind_cache): the next
  // subproblem at the same (x, y) reuses it, as the reference reuses HwNewmatrix (RIPTRM.py:686-692)
  char* big_cache = nullptr;
  int big_cache_order = 0, big_cache_batch = 0;
  int64_t big_cache_hits = 0, big_subproblems = 0;   // since the solve began (riptrm_trs_cache_stats)
  int64_t big_cg_checked = 0, big_cg_skipped = 0;    // since the context was created (riptrm_trs_skip_stats)
  void* eig_scratch = nullptr;   // riptrm_sym_eig's d / e / tau vectors (context-owned)
  size_t eig_scratch_bytes = 0;
  void* tri_grid = nullptr;      // the distributed tridiagonalisation's granules (riptrm_tri.h, context-owned)
  size_t tri_grid_bytes = 0;
  int64_t tri_fallbacks = 0;     // subproblems the tridiagonal path handed to the eigendecomposition path
};

// riptrm_trs_big.hip
int riptrm_big_service(riptrm_ctx* c, int* served);
int riptrm_big_trs_gep(riptrm_ctx* c, int dim, int batch, const double* A, int64_t lda, int64_t a_stride, const double* a,
                       int64_t ldv, const double* Delta, double tolhc, double* x, double* lam1, int32_t* kind,
                       double* mineig);
void riptrm_big_release(riptrm_ctx* c);
int riptrm_big_reset_cache(riptrm_ctx* c);
// A per-instance eigendecomposition cache keyed by the point each matrix was built at (the
// StableIdentification service): the trial point's eigensolve stores its compact eigenpairs, a
// subproblem built at exactly that point (bitwise) takes them instead of an eigensolve.
struct KeyedEigCache {
  const double* keys = nullptr;   // instance b's key at keys + b kstride, klen doubles
  int64_t kstride = 0;
  int klen = 0;
  double* cache = nullptr;        // instance b's entry at cache + b cstride (riptrm_big_kcache_doubles)
  int64_t cstride = 0;
  int mode = 0;                   // 1: every subproblem of the call is a hit; 2: store after the eigensolve
};
constexpr int RIPTRM_EIG_COMPACT_MAX = 199;   // riptrm_eig::EIG_LDS_MAX: orders with compact eigenpairs
int64_t riptrm_big_kcache_doubles(int dim, int klen);
bool riptrm_big_kcache_usable(int dim);   // the hand-written eigensolver serves dim (compact eigenpairs)
int riptrm_big_kcache_split(riptrm_ctx* c, int dim, const std::vector<int32_t>& ids, const KeyedEigCache& kc,
                            std::vector<int32_t>& hit, std::vector<int32_t>& miss);
int riptrm_big_gep_ids(riptrm_ctx* c, int dim, const int32_t* sel, int count, const double* A, int64_t lda,
                       int64_t a_stride, const double* a, int64_t ldv, const double* Delta, double tolhc, double* x,
                       double* lam1, int32_t* kind, double* mineig, bool mineig_only, bool per_instance,
                       const KeyedEigCache* kc = nullptr);


inline int fail(riptrm_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(c, expr)                                                                    \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) return fail((c), RIPTRM_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

