// Device-side structures of the SW (seed extension + CIGAR) stage.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __HIPCC__
#define SW_HD __host__ __device__
#else
#define SW_HD   // the host-compiled kernel-core tests (tests/native) include this header with g++
#endif

namespace prgpu {

// CIGAR output: every task owns a slot sized from its short-read length (cig_slot_ops;
// >= 99.7 % of 150 bp CIGARs at 15 % long-read error fit) in one pool; a CIGAR that
// outgrows its slot marks the task SW_ST_OVERFLOW and the overflow pass recomputes it
// into a spill area of the same pool, bounded by its aligned lengths (every op consumes
// at least one query or reference base).  o_cig_at[t] is where the task's ops start.
constexpr int SW_ST_OVERFLOW = 1;     // internal status, resolved before pr_sw_launch returns
SW_HD inline int cig_slot_ops(int lq) {
    const int c = (lq * 5 / 8 + 16 + 7) & ~7;   // 150 bp: 112 ops (15 % error: mean 41, max seen 79)
    return c > 16 ? c : 16;
}
SW_HD inline int cig_bound_ops(int lqq, int rlen) { return lqq + rlen + 4; }
constexpr int SW_WAVE = 64;
constexpr int SW_NBUCKET = 1024;      // task-ordering keys (query lengths <= 1000)
constexpr int PK_NB = 41 * 256;       // packed-kernel keys: band (<= 40) x query length (<= 255)
constexpr int PK_SCAN = 11 * 1024;    // scanned key range (PK_NB rounded up to the scan's 1024 x 11)
constexpr int PK_SEG = 128;           // tasks per wave (two per lane)

struct SwOptsDev {
    int a, b, o_del, e_del, o_ins, e_ins, w, pen_clip5, pen_clip3, zdrop;
    double min_score_per_base;
    int pk;      // 1: the packed two-tasks-per-lane CIGAR kernel may take tasks (penalties fit its int16 frame)
    int debug;   // timing ablations only (PRGPU_SW_DEBUG): 1 = skip backtrack, 2 = skip z stores
};

struct SwDev {
    int64_t n_task;
    int qmax;                  // longest short read in the batch
    int tmax;                  // bound on reference window rows (qmax + 4w)
    const uint8_t *sr;         // nt4 short reads
    const int64_t *sr_off;
    const uint8_t *lr;         // nt4 long reads (forward)
    const int64_t *lr_off;
    const int32_t *t_sr, *t_lr, *t_qbeg, *t_rbeg, *t_slen;
    const uint8_t *t_strand;
    // extension results (inputs of the global kernel)
    int32_t *o_qb, *o_qe, *o_rb, *o_re, *o_score, *o_truesc, *o_w;
    uint8_t *o_pass;
    // global / CIGAR results
    int32_t *o_gscore, *o_pos, *o_ncig, *o_status;
    uint32_t *o_cig;           // CIGAR pool: the slots (cig_slot prefix), then the spill area
    const int64_t *cig_slot;   // [n_task+1] prefix of the slot capacities
    int64_t *o_cig_at;         // [n_task] first op of the task's CIGAR in o_cig
    unsigned long long *spill; // [0] overflowed tasks, [1] their op bounds summed, [2] spill cursor
    int64_t spill_base;        // first op of the spill area
    int rerun;                 // sw_global_kernel: 1 = the overflow pass (ops at o_cig_at, bounded)
    uint32_t *eh_g;            // sw_global_kernel DP row in HBM (queries too long for LDS), or null
    int64_t eh_g_stride;       // dwords per block of eh_g
    int eh_g_blocks;           // blocks eh_g holds (grid of the HBM-row kernels)
    uint8_t *z;                // direction-matrix slabs, one per resident block
    int64_t z_slab;            // bytes per slab (LDS kernel)
    int64_t z_ring_slab;       // dwords per slab (register-ring kernels: rows x words x 64 lanes)
    int64_t z_pk_slab;         // PkDir entries per slab (packed kernel: rows x chunks x 64 lanes)
    int pk_chunk;              // packed CIGAR pass: segments per DP + backtrack launch pair (0: fused kernel)
    int64_t pk_nseg_bound;     // upper bound on its segments (the launch loop's extent)
    int pk_bt_grid, pk_bt_win; // backtrack kernel: grid (waves), window rows (8 or 16)
    unsigned long long *cells; // [3] canonical DP cells (extension, global, dominant launch), [3..6] pk phase cycles
    int32_t *perm;             // lane -> task order (tasks bucketed by extension lengths)
    int32_t *keyc;             // [selection] phase keys of the last listing pass (count -> scatter)
    int32_t *bucket;           // [SW_NBUCKET + 1] counting-sort scratch
    int32_t *work;             // dequeue counter for the global kernel
    int32_t *x;                // extension scratch: 2 sides x XF fields x n_task
    uint8_t *x_try;            // bit side: that side needs the second band try
    int32_t *list;             // task list of the current extension phase
    const int32_t *list_n;     // its length (device)
    int32_t *pk_bucket;        // [PK_SCAN + 1] packed-kernel key counts -> padded offsets; [PK_SCAN] = list length
    // bwa mode (tasks = every seed of the kept chains): which tasks the extension phases
    // (bit SEL_EXT) and the CIGAR phases (bit SEL_CIG) take; null = all tasks in both
    const uint8_t *sel;
    // bwa mode: the phases iterate this task list (tsel_n entries) instead of 0 .. n_task
    const int32_t *tsel;
    int64_t tsel_n;
};
constexpr uint8_t SEL_EXT = 1, SEL_CIG = 2;
SW_HD inline bool sel_ext(const SwDev &D, int64_t t) { return !D.sel || (D.sel[t] & SEL_EXT); }
SW_HD inline bool sel_cig(const SwDev &D, int64_t t) { return !D.sel || (D.sel[t] & SEL_CIG); }
SW_HD inline int64_t sel_count(const SwDev &D) { return D.tsel ? D.tsel_n : D.n_task; }
SW_HD inline int64_t sel_task(const SwDev &D, int64_t k) { return D.tsel ? (int64_t)D.tsel[k] : k; }

// HIP events around every extension DP launch of one pr_sw_launch (the extension stage's
// roofline: its DP cells over the summed launch durations); pairs (start, end)
struct SwEvPool {
    static const int CAP = 128;
    void *ev[CAP] = {};
    int n = 0;
    int dropped = 0;   // marks the full pool could not take (launches left untimed)
};

struct SwResident {
    bool loaded = false;
    int64_t n_task = 0, n_sr = 0, n_lr = 0;
    int qmax = 0;
    void *buf[80] = {};
    size_t cap[80] = {};
    // bwa mode (pr_sw_batch.t_chain): the tasks are seeds, the outputs reported alignments
    bool bwa = false;
    int64_t read_id0 = 0;
    int64_t n_aln = 0;          // reported alignments of the last launch
    int ext_rounds = 0;         // extension rounds of the last launch (mem_chain2aln resumes)
    int64_t n_ext = 0;          // seeds extended
    int64_t n_rank0 = 0;        // first seeds of the chains (the first round)
    bool cnext_ready = false;   // cnext written by the device-seed unpack (seed ranks)
    int64_t n_big = 0;          // bwa mode: reads of more than ALN_WAVE_SEEDS seeds (the lane kernels')
    void *side = nullptr;       // hipStream_t: the early final pass beside the later extension rounds
    void *side_ev[3] = {nullptr, nullptr, nullptr};   // hipEvent_t
    int64_t n_patch = 0;        // mem_patch_reg global scores computed
    // bwa mode's bookkeeping kernels of the last launch (timing events, created on first use):
    // [0, 1] each round's walk, [2, 3] each late final pass, [4, 5] the early final pass (side
    // stream), [6, 7] its complement on the main stream
    void *bt_ev[8] = {};
    float ms_walk = 0.f, ms_final = 0.f, ms_final_early = 0.f;
    int64_t cig_slots = 0;      // ops in the slots (= first spill op)
    int64_t n_overflow = 0;     // tasks of the last launch whose CIGAR went to the spill area
    float ms_ext = 0.f, ms_glob = 0.f;
    unsigned long long cells[3] = {0, 0, 0};
    float ms_glob_ring = 0.f;
    SwEvPool ext_ev;
};

// device pointers of a resident SW batch (for the SW -> consensus pipeline); in bwa mode
// the per-task arrays are the reported alignments grouped by long read (task_off)
struct SwPtrs {
    const uint8_t *sr, *lr, *strand, *pass;
    const int64_t *sr_off, *lr_off;
    const int32_t *t_sr, *t_lr, *status, *pos, *score, *ncig;
    const uint32_t *cig;
    const int64_t *cig_at;
    int64_t n_task;
    int n_sr, n_lr;
    const int64_t *task_off;    // bwa mode: [n_lr+1] alignments of long read i; else null
    int max_per_lr;             // bwa mode: most alignments on one long read
};

int sw_launch_order(const SwDev &D, const SwOptsDev &O, int phase, int32_t *out, void *stream);
int sw_launch_extend(const SwDev &D, const SwOptsDev &O, int grid_waves, int grid_pk, void *stream,
                     SwEvPool *evp = nullptr);
// side / ev_fork / ev_join / z_side (optional): the band-80 ring kernel's tasks listed and run on
// the side stream beside the packed kernel, with its own direction slabs at z_side
int sw_launch_global(const SwDev &D, const SwOptsDev &O, int grid_waves, int grid_pk, int grid_lds, int lds,
                     void *stream, void *ev_a, void *ev_b, bool pk_ordered = false, void *side = nullptr,
                     void *ev_fork = nullptr, void *ev_join = nullptr, void *z_side = nullptr, void *ev_mid = nullptr);
int sw_launch_pk_order(const SwDev &D, const SwOptsDev &O, int mode, void *stream);
int sw_pk_bt_occupancy(int win);
int sw_launch_lds(const SwDev &D, const SwOptsDev &O, int grid, int lds, void *stream);
int sw_launch_overflow(const SwDev &D, const SwOptsDev &O, int grid, int lds, void *stream);
int sw_launch_cig_compact(const uint32_t *pool, const int64_t *at, const int32_t *ncig, const int64_t *off,
                          int64_t n, uint32_t *out, void *stream);
void sw_release(SwResident &r);
// bwa mode: gather the reported alignments by long read (stable: read order inside a long read)
struct SwGather {
    const int32_t *list;        // alignment -> task
    int64_t n;
    const int32_t *t_sr, *status, *pos, *score, *ncig, *qb, *qe, *rb, *re, *truesc, *flag_in;
    const uint8_t *strand, *pass;
    const int64_t *cig_at;
    int32_t *o_sr, *o_status, *o_pos, *o_score, *o_ncig, *o_qb, *o_qe, *o_rb, *o_re, *o_truesc, *o_task, *o_lr;
    const int32_t *t_lr;
    uint8_t *o_strand, *o_pass;
    int64_t *o_cig_at;
};
int sw_launch_gather(const SwGather &G, void *stream);

}  // namespace prgpu
