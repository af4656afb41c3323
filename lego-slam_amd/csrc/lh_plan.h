// lh_plan.h — window preprocessing for the device layout (host only, no HIP).
//
// One sliding window (include/lego_ba.h lh_window) becomes:
//   * a landmark-major order of the observations, each landmark's observations in ascending pose
//     order (the reference visits edges in unordered_map order, problem.cpp:285; any order is the
//     same problem);
//   * landmarks ordered by observation span and packed into chunks whose union of observing poses
//     fits one MFMA window (<= LH_UMAX poses), chunks split into wave sub-batches (<= 8 landmarks,
//     <= 64 observations, landmark l owning the aligned lane group [l*G, l*G + k_l));
//   * the reduce plan: for every pose pair p <= q, the chunks whose slab holds a block of it.
// Two phases so the bulk arrays are written once, straight into the caller's (pinned) staging:
// plan_structure() sizes everything (O(O) scan + O(L) ordering), plan_fill() writes the arrays.
// Both run on a small thread pool; the result does not depend on the thread count.
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/lego_ba.h"
#include "lh_common.h"

namespace lh {

// Persistent worker pool: run(n, fn) calls fn(i) for i in [0, n) on the workers and the caller.
// The job hand-off is lock-free (Pool::loop); an idle worker polls the job generation briefly
// (kSpin pauses) and then sleeps on the condition variable.  Polling longer (300 us after each job,
// so that a planning pass's back-to-back jobs never wait for a wake-up) measured slower on the box's
// 16-CPU cgroup share: lh_solve's preprocessing 1.80 ms against 1.49 ms.
class Pool {
  public:
    explicit Pool(int threads);
    ~Pool();
    int size() const { return (int)workers_.size() + 1; }
    void run(int n, const std::function<void(int)>& fn);

  private:
    struct Job {
        const std::function<void(int)>* fn = nullptr;
        int n = 0;
        std::atomic<int> next{0};
    };
    static constexpr unsigned kSpin = 256;
    void loop();
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::atomic<Job*> job_{nullptr};    // the live job, nullptr once run() retires it
    std::atomic<uint64_t> gen_{0};      // bumped per job
    std::atomic<int> active_{0};        // workers that may still touch job_'s job
    std::atomic<int> sleepers_{0};
    std::atomic<bool> stop_{false};
    std::vector<int> pinned_;           // the CPU id each worker is pinned to (its use count released on destruction)
};

struct PlanCfg {
    int chunk_lm = 0;      // landmarks per chunk; 0 = auto (~512 chunks, 2 workgroups per CU)
    bool rank_invariant_pairs = false;   // P > LH_PMAX_WIN: list every pair within the 64-pose span (sharded solves)
};

struct Plan {
    // ---- sizes (plan_structure) ----
    int P = 0, L = 0, ncam = 1;
    int64_t O = 0;
    int n_chunks = 0, n_sb = 0, n_items = 0, npairs = 0;
    int n_rec = 0;                      // landmark records (8 per sub-batch)
    int64_t n_slots = 0;                // observation slots (64 per sub-batch)
    int tgroup_begin[LH_TMAX + 2] = {0};
    uint64_t fixed_mask = 0;            // bit p: pose p < 64 is fixed (fixed_bits[0])
    std::vector<uint64_t> fixed_bits;   // [(P + 63) / 64] bit p % 64 of word p / 64: pose p is fixed
    std::vector<uint16_t> pair_list;    // [2 npairs] (p, q), p <= q, of each reduced-system block
    // the blocks by block row (the PCG's S p, k_ctrl_p): row p holds, in ascending column q, entry
    // (b << 13) | (q << 1) | t for block b = pair (min(p, q), max(p, q)), t = 1 where it is read transposed
    std::vector<int32_t> brow_ptr;      // [P + 1]
    std::vector<uint32_t> brow_ent;     // [2 npairs - P]
    // ---- internal (reused across windows) ----
    std::vector<int64_t> lm_ptr;        // [L+1] CSR over landmarks
    std::vector<int64_t> csr;           // [O] window obs, landmark-major, ascending pose
    std::vector<uint64_t> lm_mask;      // [L] observing-pose mask, bit i = pose lm_base + i
    std::vector<int32_t> lm_base;       // [L] first observing pose
    std::vector<int32_t> order;         // [L_act] landmarks with edges, span order
    std::vector<uint64_t> ord_mask;     // [L_act] lm_mask / lm_base / log2 lane group, in span order
    std::vector<int32_t> ord_base;
    std::vector<uint8_t> ord_lg;
    std::vector<int32_t> chunk_lm0;     // [n_chunks + 1] chunk c owns order[chunk_lm0[c] .. chunk_lm0[c+1])
    std::vector<uint64_t> chunk_mask;   // [n_chunks] union pose mask, bit i = pose chunk_base + i
    std::vector<int32_t> chunk_base;    // [n_chunks]
    std::vector<int32_t> chunk_sb0;     // [n_chunks + 1] sub-batch prefix (chunks in T order)
    std::vector<int32_t> corder;        // [n_chunks] launch order (grouped by T) -> chunk
    std::vector<int32_t> sb_lm0;        // [n_sb + 1] sub-batch -> first position in order[]
    std::vector<uint8_t> sb_lg;         // [n_sb]
    std::vector<uint32_t> pair_ptr;     // [npairs + 1]
    std::vector<uint32_t> chunk_ib;     // [n_chunks + 1] first item of each chunk (launch order)
    double t_stage[8] = {0};            // diagnostic: ms at plan_structure's stage ends (lhp_plan_stages)
};

struct PlanOut {
    lh_chunk* chunks;        // [n_chunks]
    lh_subbatch* sbs;        // [n_sb]
    uint32_t* meta;          // [n_slots]
    float* uv;               // [2 n_slots] pixels as float: toVec2 of cv::KeyPoint::pt (algorithm.h:37),
                             // so every measurement is a float (plan_structure rejects one that is not)
    int32_t* obs_perm;       // [n_slots] slot -> window obs (-1: padding)
    int32_t* lm_perm;        // [n_rec] record -> window landmark (-1: padding)
    uint32_t* items;         // [n_items] per chunk (launch order), per slot pair (s <= t): its pair row
    uint16_t* pair_pq;       // [2 npairs]
    uint32_t* rsmap;         // [npairs * 36]
    double* lm_xyz;          // [3 L] copy of the window's positions (nullptr: not wanted)
};

// lh_status.  LH_E_BADARG for out-of-range indices, LH_E_UNSUPPORTED outside the envelope
// (DESIGN.md "Limits"), LH_E_EMPTY mirrors problem.cpp:157-161.
int plan_structure(const lh_window* w, const PlanCfg& cfg, bool allow_empty, Plan& pl, Pool* pool);
// on_slots(slot_begin, slot_end), if given, is called on the calling thread each time the observation
// slots [slot_begin, slot_end) (meta, uv, obs_perm) are final, in ascending order, so the caller can
// start copying them while the rest is filled; `batches` splits the chunk pass for that.
using SlotsReady = void (*)(void* user, int64_t slot_begin, int64_t slot_end);
// Returns LH_OK (the window was validated by plan_structure).
int plan_fill(const lh_window* w, const Plan& pl, const PlanOut& out, Pool* pool, SlotsReady on_slots = nullptr,
              void* user = nullptr, int batches = 1);

}  // namespace lh
