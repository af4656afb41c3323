// lh_common.h — data layout shared by the HIP kernels and the host side of
// liblego_ba.so.  See DESIGN.md "Data layout in HBM".
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#define LH_HD __host__ __device__
#else
#define LH_HD
#endif

// ---- envelope ---------------------------------------------------------------
#define LH_PMAX 21            // poses per window solved in LDS (reduced system n = 6P <= 126, k_ctrl)
#define LH_PMAX_WIN 64        // the dense packed reduced-system layout (every pose pair a block) and the
                              // LDL^T in global memory (k_ctrl_g, 6P <= 384 rows)
#define LH_PMAX_ANY 256       // poses per window at all (PCG on the block-sparse reduced system, k_ctrl_p);
                              // a landmark's observing poses must lie within 64 consecutive ones
#define LH_UMAX 16            // distinct poses in one chunk window (6U <= 96 rows); the reference window is
                              // 15 keyframes (map.h:82), so any landmark of it fits one chunk window
#define LH_TMAX 6             // 16-row MFMA tiles per window side
#define LH_SB_LM 8            // landmarks per sub-batch (one wave)
#define LH_SB_OBS 64          // observations per sub-batch (one per lane)
#define LH_WAVES 4            // waves per k_lin workgroup
#define LH_TASKS 33           // per-pose values a sub-batch emits: Hpp(21) bp(6) bsd(6)
#define LH_MAX_CAMS 4
#define LH_TRACE 64
#define LH_LAD 16             // lambda-ladder rungs at most (one controller workgroup each, lh_ctrl.lad)
#define LH_NPAD 128           // reduced system padded size (LDS LDLT)
#define LH_IMG_AS (LH_NPAD + 2)                 // k_ctrl's LDS row stride (doubles)
#define LH_IMG_SZ ((LH_NPAD + 1) * LH_IMG_AS)   // k_ctrl's LDS system image: NP rows of S + the rhs row (doubles)

// pair row (k_lin -> k_reduce): S block landmark part (36) | the pose's 33 sums (diagonal pairs) | pad
#define LH_ROW 72

// slab scalars
#define LH_SC_CHI2 0          // sum rho0 (not halved)
#define LH_SC_SCALE 1         // landmark part of dx^T(lambda dx + b)
#define LH_SC_NDEG 2          // rank-deficient H_ll landmarks
#define LH_SC_MAXD 3          // max |H_ll diag| (a max, not a sum)

// per-landmark record (one 128-B line, double-buffered committed/candidate):
// X (3) | Cholesky of H_ll with reciprocal diagonal {1/L00, L10, 1/L11, L20, L21, 1/L22} (6) |
// b_l (3) | diag H_ll (3) | pad.  A sub-batch owns 8
// consecutive records, so one wave moves its landmarks with one 16-B access per lane.
#define LH_REC 16
#define LH_REC_X 0
#define LH_REC_L 3
#define LH_REC_B 9
#define LH_REC_HD 12

// Pose state is estimate_ itself: a row-major [R | t] matrix per pose (12 doubles,
// VertexPose stores the 4x4, lego_types.h:37,57).  Every use converts it to
// Sophus' (quaternion, t) as SE3(estimate_) does (lego_types.h:211,229); the
// per-trial pose table caches those conversions:
//   per (pose, cam), LH_PT doubles:  q_T[4] t_T[3] | q_et[4] t_et[3] (ext*T) | R_T[9] | pad
//   per cam, LH_EXT doubles:         q_e[4] t_e[3] | R_e[9]
#define LH_PT 24
#define LH_PT_QT 0
#define LH_PT_TT 4
#define LH_PT_QET 7
#define LH_PT_TET 11
#define LH_PT_RT 14
#define LH_EXT 16

// reduced-system element map (k_ctrl scatter): row | col << 9 | diagonal-block flag << 18
#define LH_RSMAP(r, c, d) ((uint32_t)(r) | ((uint32_t)(c) << 9) | ((d) ? (1u << 18) : 0u))
#define LH_RSMAP_ROW(m) ((m) & 0x1FFu)
#define LH_RSMAP_COL(m) (((m) >> 9) & 0x1FFu)
#define LH_RSMAP_DIAG(m) ((m) >> 18)

// obs meta packing
#define LH_META(pose, cam, slot, lms) ((uint32_t)(pose) | ((uint32_t)(cam) << 12) | ((uint32_t)(slot) << 16) | ((uint32_t)(lms) << 20) | LH_META_VALID)
#define LH_META_VALID (1u << 23)
#define LH_META_POSE(m) ((m) & 0xFFFu)
#define LH_META_CAM(m) (((m) >> 12) & 0xFu)
#define LH_META_SLOT(m) (((m) >> 16) & 0xFu)
#define LH_META_LMS(m) (((m) >> 20) & 0x7u)

struct lh_chunk {
    uint32_t sb_begin, sb_end;   // sub-batch range
    uint8_t U, T, pad0, pad1;
    uint16_t pose[LH_UMAX];      // window slot -> pose
    uint32_t item_base;          // the chunk's U(U+1)/2 entries of the row map (items[])
};

// A sub-batch is one wave's unit of work: n_lm landmarks, landmark l owning the
// aligned lane group [l*G, l*G + k_l) of the sub-batch's 64 observation slots
// (slots sb*64 .. sb*64+63; unused slots carry a meta word without LH_META_VALID).
struct lh_subbatch {
    uint32_t lm_begin;
    uint8_t n_lm, lg;      // landmarks, log2(G) lanes per landmark
    uint16_t pad;
};

// reduced-system buffer layout (one per state buffer)
struct lh_rs_layout {
    int npairs, off_S, off_bs, off_bp, off_hd, off_sc, off_bsc, total;
};

// npairs: the blocks of S (every pose pair up to LH_PMAX_WIN poses, P (P + 1) / 2; past it the pairs
// a landmark couples plus every diagonal block)
LH_HD static inline lh_rs_layout lh_rs_make(int P, int npairs) {
    lh_rs_layout L;
    L.npairs = npairs;
    L.off_S = 0;
    L.off_bs = L.npairs * 36;
    L.off_bp = L.off_bs + 6 * P;
    L.off_hd = L.off_bp + 6 * P;
    L.off_sc = L.off_hd + 6 * P;
    // a batch's per-rung chi2 and gain scale, last: in the same chunk of a ring all-reduce as the
    // single-trial scalars, so they are summed over the ranks in the same order
    L.off_bsc = L.off_sc + 8;
    L.total = L.off_bsc + 2 * LH_LAD;
    return L;
}

// LM controller state (device resident, mirrors Problem's members problem.h:157-165)
struct lh_ctrl {
    double chi, lambda, ni, last_chi, chi2_initial;
    int32_t iter, false_cnt, trials, accepted, done, cur, trace_len;
    int32_t nonpd;             // rank-deficient H_ll landmarks at the initial linearisation
    int32_t pcg_iters;         // PCG iterations summed over the solve's trials
    int32_t evo;               // the next trial only evaluates (the final LM iteration, or after a rejection)
    int32_t evo_seq[2];        // trial seq's evo at [seq & 1]: written by the previous chain's decision, so the
                               // kernels after this trial's decision (k_reduce's blocks, k_ctrl) still read it
    int32_t acc_hist[2];       // trial seq's LM decision (accepted) at [seq & 1]: read by its controller, and by
                               // the next trial's k_reduce when it commits the staged system (commit_in_reduce)
    int32_t done_seq;          // the trial whose decision stopped the loop (its controller raises the host's done)
    int32_t relin;             // an evaluate-only trial was accepted outside the final iteration: the next chain
                               // (k_lin, k_reduce, k_ctrl) linearises the committed state instead of a trial
    int32_t seq_last;          // the last chain (trial or re-linearisation) a live decision was taken on
    // The lambda ladder: a controller that factors a system may also factor it at the lambdas
    // the next rejections would try (lambda *= ni, ni *= 2; STRATEGY1 min(11 lambda, 1e7): problem.cpp:550-551,
    // :576), one workgroup per rung, so a rejection whose rung exists needs no factor (lskip).
    int32_t lad;               // the rung the pending step (dxp + lad * n, spose_l[lad]) belongs to
    int32_t lad_n;             // rungs the last factoring controller built (1: the step alone)
    int32_t lskip;             // this chain's decision was a rejection onto a built rung: its controller exits
    int32_t lskips;            // such decisions in this solve (lh_debug_ladder)
    int32_t dec_tag;           // seq + 1 once workgroup 0 of a controller that decides itself has decided chain seq
                               // (its rung workgroups wait for it; zeroed with the controller at every restart)
    // Batched evaluation of a rejection run: after a rejection, when the next trials only evaluate
    // and their steps are built rungs, one chain's k_lin evaluates consecutive rungs (their count rides above the low
    // byte of the evo words, evo and evo_seq) and k_reduce (or the controller after an exchange) takes their
    // decisions in order.  An acceptance among them is linearised by the next chain, a full trial at that rung whose
    // decision is the acceptance already taken (retrial).
    int32_t retrial;           // the next chain re-runs the accepted rung as a full trial; its decision only commits
    int32_t rho_sel;           // per-edge rho0 "as last evaluated": rung buffer (0: the ordinary one)
    int32_t nbatches;          // batches decided in this solve (lh_debug_batch)
    int32_t nretrials[2];      // their acceptances: [0] re-run as a full trial, [1] that also stopped the loop
    int32_t nofactor;          // the last decision left nothing to factor (relin | lskip | retrial: ladder_read's one word)
    int32_t lad_its[LH_LAD];   // PCG iterations of each rung's solve (counted when the rung is used)
    double spose_l[LH_LAD];    // pose part of each rung's gain denominator (isGoodStepInLM's scale)
    double trace_chi[LH_TRACE], trace_lambda[LH_TRACE];
};

// The host-visible words (pinned, mapped; written by ctrl_lm_step): done (the LM loop stopped), the
// progress word, and the solve's summary, written before done is raised, so a solve that returns no
// arrays ends when the host sees done: no copy of lh_ctrl behind the last kernel, no stream sync.
struct lh_host_words {
    int32_t done, progress;
    int32_t iter, trials, accepted, trace_len, nonpd, pcg_iters;
    double chi2_initial, chi, lambda;
    double trace_chi[LH_TRACE], trace_lambda[LH_TRACE];
};

struct lh_params {
    int32_t P, n, ncam, max_iters, max_trials, strategy, guard, lambda_given;
    int32_t npairs;         // blocks of the reduced system (lh_rs_make)
    int32_t ext_rot_identity;   // bit c: camera c's extrinsic rotation is exactly the identity
    int32_t ext_identity;   // bit c: camera c's extrinsic is exactly the identity
    int32_t solver;         // 0 LDL^T (Eigen LDLT, problem.cpp:420), 1 PCG (problem.cpp:422, :584-614)
    int32_t gate_mode;      // 0 reference Huber gate (base_edge.cpp:55); 1 diagnostic (residue taken as 0)
    int32_t no_evo;         // 1: every trial linearises in full (diagnostic A/B of ctrl.evo; env LH_NO_EVO)
    int32_t eval_first;     // 1: a trial after a rejection in its iteration only evaluates (ctrl.evo); an accepted
                            //    one is linearised by the next chain (ctrl.relin).  Env LH_NO_EVAL_FIRST: 0
    double huber_delta, stop_dchi2, tau, lambda_cap, lambda_init;
    double pcg_tol;         // PCG stop: ||r|| <= pcg_tol ||b|| (reference 1e-6, problem.cpp:597)
    int32_t pcg_max_it;     // PCG cap (<= 0: 2 * rows, problem.cpp:422)
    int32_t precision;      // lh_precision: 0 fp64 throughout, 1 fp32 per-edge residual/Jacobians (k_lin<T, TRIAL, true>)
    int32_t dec_in_reduce;  // 1: k_reduce's scalar block takes the LM decision (one rank; k_ctrl, k_ctrl_b)
    int32_t nd_a, nd_s, nd_long_first, nd_steps;   // k_ctrl's two-chain split (lh_ctrl_nd_plan; nd_steps 0: off)
    int32_t commit_in_reduce;   // 1: k_reduce copies an accepted trial's staged blocks to the committed system
                                //    before it overwrites them (k_ctrl_b: no one-CU copy of a large system)
    int32_t img;            // 1: k_reduce writes S's lower triangle and b_s straight into k_ctrl's LDS layout
                            //    (img[0] staged, img[1] committed; one rank, P <= LH_PMAX, one-chain LDL^T)
    int32_t band_narrow;    // 1: every row's envelope starts at most 56 rows above its 8-row block (k_ctrl_b's back
                            //    substitution holds one row per lane: a 64-row window)
    int32_t bimg;           // 1: k_reduce writes S's lower band straight into k_ctrl_b's band image (one rank, banded
                            //    LDL^T): the stream loaders read it without the block-index round trip
    int32_t band_lu;        // 1: some banded LDL^T step needs more than 11 unit waves: the stream loaders take units
    int32_t ladder;         // lambda-ladder rungs a factoring controller builds (1: off; k_ctrl, k_ctrl_b with
                            //    dec_in_reduce; env LH_NO_LADDER=1: 1)
    int32_t ladder_eager;   // 1: every factor builds the ladder; 0: only a factor after a rejection (env LH_LADDER_LAZY)
    int32_t lad_stride;     // doubles of a rung's global scratch (k_ctrl_g: its gA; k_ctrl_p: its row copy of S)
    int32_t batch;          // rejection runs evaluated in batches of rungs (one rank, k_reduce decides; env LH_NO_BATCH)
    int32_t n_chunks;       // k_lin chunks of the window (the per-rung chunk scalars' stride)
    double K[4];
};

// ---- the controllers' work units ------------------------
// The reduced system is factored in natural pose order, so its nonzeros stay within the envelope of
// S (row r's first nonzero column: the first pose any chunk couples with r's pose).  Step t of the
// blocked LDL^T eliminates block column 8t; a 16-row tile row I takes part iff its envelope reaches
// that column: tile_fcb[I] (its first nonzero 8-column block) <= t.  Per step, the trailing tiles of
// the active tile rows are dealt to the unit waves (wave 0 runs the diagonal tile and the next block's
// factor): one tile per unit when they fit, else half tile rows.  Unit word (u16) of wave w at step t,
// units[w * nstep_max + t]: bit 15 valid, bit 14 store L^T and the rhs row, bits 0-2 tile row, 3-5
// first tile column, 6-9 end tile column (exclusive), all relative to g0 = (8t + 8) / 16, the tile
// holding the next diagonal block.  Wave 0's word: bit 15 = its diagonal tile is active.
// Returns the most units any step needed (more than the waves given: the table is incomplete).
#define LH_UNIT_VALID 0x8000u
#define LH_UNIT_STORE 0x4000u
#define LH_NSTEP (LH_NPAD / 8)
LH_HD static inline uint16_t lh_unit(int I, int jb0, int jb1, bool store) {
    return (uint16_t)(LH_UNIT_VALID | (store ? LH_UNIT_STORE : 0u) | (uint32_t)I | ((uint32_t)jb0 << 3) | ((uint32_t)jb1 << 6));
}
LH_HD static inline int lh_ctrl_units(int n, const int32_t* tile_fcb, const int* order, int nwaves, int nstep_max,
                                      uint16_t* units) {
    const int NE = (n + 15) & ~15, nb = (n + 7) & ~7, gl = NE / 16 - 1;
    int worst = 0;
    for (int i = 0; i < 16 * nstep_max; ++i) units[i] = 0;
    for (int t = 0; t < nstep_max; ++t) {
        const int m0 = 8 * t + 8;
        if (m0 >= nb) break;
        const int g0 = m0 >> 4;
        const bool act0 = tile_fcb[g0] <= t;
        if (act0) units[t] = (uint16_t)LH_UNIT_VALID;
        uint16_t item[16];
        int cost[16], ni = 0, tiles = 0, rows = 0;
        int jmin[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int gend = (gl < g0 + 7) ? gl : g0 + 7;   // relative indices fit 3 bits
        for (int I = g0 + 1; I <= gend; ++I) {
            if (tile_fcb[I] > t) continue;
            int j = g0;
            while (j < I && tile_fcb[j] > t) ++j;
            jmin[I - g0] = j;
            tiles += I - j + 1;
            ++rows;
        }
        for (int I = gend + 1; I <= gl; ++I)   // a band wider than 8 tile rows: not representable
            if (tile_fcb[I] <= t) worst = 99;
        const bool per_tile = tiles + (act0 ? 1 : 0) <= nwaves;
        const int need = per_tile ? tiles + (act0 ? 1 : 0) : 2 * rows + (act0 ? 1 : 0);
        worst = need > worst ? need : worst;
        if (act0) { item[ni] = lh_unit(0, 0, 0, true); cost[ni++] = 6; }
        for (int I = g0 + 1; I <= gend; ++I) {
            if (tile_fcb[I] > t) continue;
            const int j0 = jmin[I - g0], nt = I - j0 + 1, ir = I - g0, jr = j0 - g0;
            if (per_tile) {
                for (int J = 0; J < nt; ++J) { item[ni] = lh_unit(ir, jr + J, jr + J + 1, J == 0); cost[ni++] = J == 0 ? 8 : 6; }
            } else if (nt == 1) {
                item[ni] = lh_unit(ir, jr, jr + 1, true); cost[ni++] = 8;
            } else {
                const int split = (nt + 1) >> 1;
                item[ni] = lh_unit(ir, jr, jr + split, true); cost[ni++] = 6 + 2 * split;
                item[ni] = lh_unit(ir, jr + split, jr + nt, false); cost[ni++] = 4 + 2 * (nt - split);
            }
            if (ni > 14) break;
        }
        for (int a = 1; a < ni; ++a)   // stable insertion sort, cost descending
            for (int b = a; b > 0 && cost[b] > cost[b - 1]; --b) {
                const int c = cost[b]; cost[b] = cost[b - 1]; cost[b - 1] = c;
                const uint16_t u = item[b]; item[b] = item[b - 1]; item[b - 1] = u;
            }
        for (int i = 0; i < ni && i < nwaves; ++i) units[order[i] * nstep_max + t] = item[i];
    }
    return worst;
}
// k_ctrl: all 15 waves take units, wave 0's SIMD-mates (4, 8, 12) last
#define LH_ORDER_CTRL {1, 2, 3, 5, 6, 7, 9, 10, 11, 13, 14, 15, 4, 8, 12}
// k_ctrl_b: waves 12-15 stream tile rows into the window; a step needing more than 11 units gives the rest
// to them (their loads and window writes are a few instructions per step from the band image), wave 0's
// SIMD-mate 12 last
#define LH_ORDER_BAND {1, 2, 3, 5, 6, 7, 9, 10, 11, 4, 8, 13, 14, 15, 12}
#define LH_BAND_UNIT_WAVES 15   // 11 unit waves, then the 4 stream loaders (k_ctrl_b<true>)

// k_ctrl_b's band image (prm.bimg): tile row I (rows 16 I .. 16 I + 15) holds columns 16 (I - 7) .. 16 I + 15,
// 128 per row, the order k_ctrl_b's stream loaders read (a banded window's rows start at or after column
// 16 I - 104, lh_host.cpp); two copies (staged, committed) of ceil16(6P) / 16 tile rows each
#define LH_BIMG_TR (16 * 128)
LH_HD static inline int lh_bimg_idx(int r, int c) {
    const int I = r >> 4;
    return I * LH_BIMG_TR + (r & 15) * 128 + (c - 16 * (I - 7));
}
LH_HD static inline bool lh_bimg_in(int r, int c) {
    const int o = c - 16 * ((r >> 4) - 7);
    return c <= r && o >= 0 && o < 128;
}

// ---- the one-shot peer-write exchange (LH_COMM_P2P) ---------------------------
// Every rank owns one exchange buffer, IPC-mapped into every peer: [2 parities][world slots][slot doubles], then
// [2 parities][world] 64-bit arrival tags.  Per LM trial each rank writes its partial reduced system into slot
// `rank` of every rank's buffer (its own included) and then, behind a system-scope release, its tag; each rank
// waits for all tags of the trial in its own buffer and sums the slots in rank order.  Tags are (solve << 32) |
// (chain + 1): a tag of an earlier chain or solve never matches.
#define LH_P2P_MAX 16
struct lh_peers {
    double* p[LH_P2P_MAX];   // every rank's exchange buffer, mapped into this process (p[rank]: its own)
};

// k_ctrl_b's per-window tables (bblk null: no banded controller for this window)
// The restart of a resident solve, done by the initial linearisation's block 0 (k_lin<T, false>): controller
// zeroed, both pose and pose-table buffers from their initial copies, the step zeroed; its chunks read the
// landmarks straight from the window (lm_perm, lm_in) and the initial tables from ptab_init.
struct lh_reset_args {
    const int32_t* lm_perm;    // record -> window landmark (-1: padding)
    const double* lm_in;       // [L][3] the uploaded landmark positions
    const double* qt_init;     // [2][P][12] initial poses (both slots)
    const double* ptab_init;   // [2][P * ncam * LH_PT] initial pose tables (both slots)
    int nqt, nptab, ndxp;
};

struct lh_band_args {
    const int32_t* bblk;     // [P * 64] block of pose pair (p, p + d), -1 if absent
    const uint16_t* units;   // [16 waves][6 LH_PMAX_ANY / 8 steps] unit words
    double* Lg;              // [ceil16(6P)][128] L rows
    double* NDg;             // [steps][64] ND per block
};

// the two-chain order of lh_ctrl_nd_plan as arithmetic (k_ctrl: no tables): the position of pose p, and
// the pose at position x
LH_HD static inline int lh_nd_pos(int p, int P, int a, int s, int long_first) {
    const int b = P - a - s, nlong = long_first ? a : b, nshort = long_first ? b : a;
    const bool inA = p < a, inB = p >= a + s;
    const bool inLong = long_first ? inA : inB, inShort = long_first ? inB : inA;
    const int first = inA ? 0 : (inB ? a + s : a);
    return inLong ? p - first : (inShort ? nlong + (p - first) : nlong + nshort + (p - a));
}
LH_HD static inline int lh_nd_nat(int x, int P, int a, int s, int long_first) {
    const int b = P - a - s, nlong = long_first ? a : b, nshort = long_first ? b : a;
    if (x < nlong) return long_first ? x : a + s + x;
    if (x < nlong + nshort) return long_first ? a + s + (x - nlong) : x - nlong;
    return a + (x - nlong - nshort);
}

// ---- k_ctrl's two-chain schedule (nested dissection of a banded S) ------------------
// Poses split as [A | S | B] in natural order, A and B decoupled (no chunk window holds poses of both:
// every B pose's envelope starts at or after A's end).  In the order [long part, short part, S] the
// LDL^T of the two parts are independent chains (chain 0: the long part's blocks then S's; chain 1:
// the short part's), run concurrently by wave 0 and wave 1, one barrier per step; both update S.
// A step's work units may then apply both chains' current blocks (sources): unit word bits 0-2 tile row,
// 3-5 first tile column, 6-9 end tile column (absolute tiles), 10-11 source mask, 12-13 store mask
// (L^T and the rhs row), 15 valid.  Wave 0's / wave 1's word: the sources of its next block's diagonal
// tile.  chain[c][t]: the block chain c eliminates at step t (-1: none).
#define LH_ND_SRC0 0x0400u
#define LH_ND_STORE0 0x1000u
struct lh_ctrl_nd {
    int nsteps;                       // 0: no worthwhile split (run the one-chain schedule)
    int a, s, long_first;             // [A | S | B]: A = poses [0, a), S = [a, a + s); the long part first
    int8_t chain[2][LH_NSTEP + 1];
    uint8_t pos[LH_PMAX];             // natural pose -> position in the factor order
    uint16_t units[16 * LH_NSTEP];
};
LH_HD static inline uint16_t lh_nd_unit(int I, int jb0, int jb1, int src, int store) {
    return (uint16_t)(LH_UNIT_VALID | (uint32_t)I | ((uint32_t)jb0 << 3) | ((uint32_t)jb1 << 6) | ((uint32_t)src << 10) |
                      ((uint32_t)store << 12));
}
// pf[p]: the first pose coupled with pose p (p's envelope).  Fills nd; returns nd.nsteps.
static inline int lh_ctrl_nd_plan(int P, const int* pf, lh_ctrl_nd& nd) {
    nd.nsteps = 0;
    const int n = 6 * P, NE = (n + 15) & ~15, NB = ((n + 7) & ~7) / 8, NT = NE / 16;
    if (P < 12 || P > LH_PMAX) return 0;
    int best = NB - 2, ba = -1, bs = -1, blong_first = 1;
    for (int a = 4; a < P; a += 4)
        for (int b = 4; a + b < P; b += 4) {
            const int s = P - a - b;
            bool dec = true;                              // B's envelope must not reach A
            for (int q = a + s; q < P && dec; ++q) dec = pf[q] >= a;
            if (!dec) continue;
            const int nl = 6 * (a > b ? a : b) / 8, ns = 6 * (a > b ? b : a) / 8, nS = NB - nl - ns;
            if (ns >= nl || nS < 1) continue;
            if (nl + nS < best) { best = nl + nS; ba = a; bs = s; blong_first = a > b; }
        }
    if (ba < 0) return 0;
    const int a = ba, s = bs, b = P - a - s;
    const int nlong = blong_first ? a : b, nshort = blong_first ? b : a;
    nd.a = a; nd.s = s; nd.long_first = blong_first;
    for (int p = 0; p < P; ++p) nd.pos[p] = (uint8_t)lh_nd_pos(p, P, a, s, blong_first);
    int nat[LH_PMAX];                                     // position -> natural pose
    for (int p = 0; p < P; ++p) nat[nd.pos[p]] = p;
    // block-level structure in the factor order, then the symbolic fill of the elimination
    bool nz[LH_NSTEP][LH_NSTEP];
    for (int i = 0; i < NB; ++i)
        for (int k = 0; k < NB; ++k) {
            bool v = false;
            for (int r = 8 * i; r < 8 * i + 8 && r < n && !v; ++r)
                for (int c = 8 * k; c < 8 * k + 8 && c < n && !v; ++c) {
                    const int p = nat[r / 6], q = nat[c / 6], hi = p > q ? p : q, lo = p > q ? q : p;
                    v = lo >= pf[hi];
                }
            nz[i][k] = v && i > k;
        }
    for (int k = 0; k < NB; ++k)
        for (int i = k + 1; i < NB; ++i)
            if (nz[i][k])
                for (int j = k + 1; j < i; ++j)
                    if (nz[j][k]) nz[i][j] = true;
    auto tnz = [&](int I, int k) {
        return (2 * I > k && 2 * I < NB && nz[2 * I][k]) || (2 * I + 1 > k && 2 * I + 1 < NB && nz[2 * I + 1][k]);
    };
    const int nl_blk = 6 * nlong / 8, ns_blk = 6 * nshort / 8;
    for (int c = 0; c < 2; ++c)
        for (int t = 0; t <= LH_NSTEP; ++t) nd.chain[c][t] = -1;
    int T = 0;
    for (int k = 0; k < nl_blk; ++k) nd.chain[0][T++] = (int8_t)k;
    for (int k = nl_blk + ns_blk; k < NB; ++k) nd.chain[0][T++] = (int8_t)k;
    for (int k = 0; k < ns_blk; ++k) nd.chain[1][k] = (int8_t)(nl_blk + k);
    for (int i = 0; i < 16 * LH_NSTEP; ++i) nd.units[i] = 0;
    // SIMD 2 and 3's waves first, then wave 1's SIMD-mates, then wave 0's
    const int order[14] = {2, 3, 6, 7, 10, 11, 14, 15, 5, 9, 13, 4, 8, 12};
    for (int t = 0; t < T; ++t) {
        int src_blk[2] = {nd.chain[0][t], nd.chain[1][t]};
        // the chains' next diagonal tiles
        int dg[2] = {-1, -1};
        for (int c = 0; c < 2; ++c) {
            const int nx = nd.chain[c][t + 1];
            if (nx < 0 || src_blk[c] < 0) continue;
            dg[c] = nx >> 1;
            if (c == 1 && dg[0] == dg[1]) return 0;   // waves 0 and 1 would update one tile
            int m = 0;
            for (int q = 0; q < 2; ++q)
                if (src_blk[q] >= 0 && tnz(dg[c], src_blk[q])) m |= 1 << q;
            nd.units[(c == 0 ? 0 : 1) * LH_NSTEP + t] = m ? lh_nd_unit(dg[c], dg[c], dg[c] + 1, m, 0) : 0;
        }
        uint16_t item[64];
        int ni = 0;
        auto mask_of = [&](int I, int J) {
            int m = 0;
            for (int q = 0; q < 2; ++q) {
                const int k = src_blk[q];
                if (k >= 0 && tnz(I, k) && tnz(J, k)) m |= 1 << q;
            }
            return m;
        };
        auto store_of = [&](int I) {
            int m = 0;
            for (int q = 0; q < 2; ++q) {
                const int k = src_blk[q];
                if (k >= 0 && tnz(I, k)) m |= 1 << q;
            }
            return m;
        };
        // the step's tiles in pieces of at most L consecutive tiles of one tile row (a chain's diagonal tile
        // breaks a run), the row's L^T / rhs store a unit of its own or (merge) riding on the row's first
        // piece: the smallest L (stores separate first) whose units fit the 14 unit waves
        int cost[64];
        bool fit = false;
        for (int L = 1; L <= 8 && !fit; ++L)
            for (int merge = 0; merge < 2 && !fit; ++merge) {
                ni = 0;
                bool over = false;
                for (int I = 0; I < NT && !over; ++I) {
                    const int st = store_of(I);
                    bool stored = false;
                    int j0 = -1, jm = 0, jl = -1;
                    auto close = [&]() {
                        if (j0 < 0) return;
                        const int stm = (merge && !stored) ? st : 0;
                        stored = stored || (merge && st);
                        const int ns = (jm & 1) + (jm >> 1), nst = ((jm | stm) & 1) + ((jm | stm) >> 1);
                        if (ni >= 60) { over = true; return; }
                        cost[ni] = 4 * nst + 2 * ns * (jl + 1 - j0) + (stm ? 2 : 0);
                        item[ni++] = lh_nd_unit(I, j0, jl + 1, jm, stm);
                        j0 = -1; jm = 0;
                    };
                    for (int J = 0; J <= I; ++J) {
                        const bool diag = (J == I) && (I == dg[0] || I == dg[1]);
                        const int m = diag ? 0 : mask_of(I, J);
                        if (!m) { close(); continue; }
                        if (j0 >= 0 && (jl != J - 1 || J - j0 >= L)) close();
                        if (j0 < 0) j0 = J;
                        jm |= m; jl = J;
                    }
                    close();
                    if (st && !stored) {
                        if (ni >= 60) { over = true; break; }
                        cost[ni] = 4 * ((st & 1) + (st >> 1)) + 2;
                        item[ni++] = lh_nd_unit(I, 0, 0, st, st);
                    }
                }
                fit = !over && ni <= 14;
            }
        if (!fit) return 0;
        for (int a = 1; a < ni; ++a)   // stable insertion sort, cost descending: the heaviest on the freest SIMDs
            for (int b = a; b > 0 && cost[b] > cost[b - 1]; --b) {
                const int c = cost[b]; cost[b] = cost[b - 1]; cost[b - 1] = c;
                const uint16_t u = item[b]; item[b] = item[b - 1]; item[b - 1] = u;
            }
        for (int i = 0; i < ni; ++i) nd.units[order[i] * LH_NSTEP + t] = item[i];
    }
    nd.nsteps = T;
    return T;
}
