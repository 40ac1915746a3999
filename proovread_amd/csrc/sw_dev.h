// Device-side structures of the SW (seed extension + CIGAR) stage.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace prgpu {

constexpr int SW_MAXCIG = 128;   // CIGAR ops per task (PR_SW_MAXCIG)
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
    uint32_t *o_cig;           // n_task * SW_MAXCIG
    uint8_t *z;                // direction-matrix slabs, one per resident block
    int64_t z_slab;            // bytes per slab (LDS kernel)
    int64_t z_ring_slab;       // dwords per slab (register-ring kernels: rows x words x 64 lanes)
    int64_t z_pk_slab;         // PkDir entries per slab (packed kernel: rows x chunks x 64 lanes)
    unsigned long long *cells; // [3] canonical DP cells (extension, global, dominant launch), [3..6] pk phase cycles
    int32_t *perm;             // lane -> task order (tasks bucketed by extension lengths)
    int32_t *bucket;           // [SW_NBUCKET + 1] counting-sort scratch
    int32_t *work;             // dequeue counter for the global kernel
    int32_t *x;                // extension scratch: 2 sides x XF fields x n_task
    uint8_t *x_try;            // bit side: that side needs the second band try
    int32_t *list;             // task list of the current extension phase
    const int32_t *list_n;     // its length (device)
    int32_t *pk_bucket;        // [PK_SCAN + 1] packed-kernel key counts -> padded offsets; [PK_SCAN] = list length
};

struct SwResident {
    bool loaded = false;
    int64_t n_task = 0, n_sr = 0, n_lr = 0;
    int qmax = 0;
    void *buf[32] = {};
    size_t cap[32] = {};
    float ms_ext = 0.f, ms_glob = 0.f;
    unsigned long long cells[3] = {0, 0, 0};
    float ms_glob_ring = 0.f;
};

// device pointers of a resident SW batch (for the SW -> consensus pipeline)
struct SwPtrs {
    const uint8_t *sr, *lr, *strand, *pass;
    const int64_t *sr_off, *lr_off;
    const int32_t *t_sr, *t_lr, *status, *pos, *score, *ncig;
    const uint32_t *cig;
    int64_t n_task;
    int n_sr, n_lr;
};

int sw_launch_order(const SwDev &D, const SwOptsDev &O, int phase, int32_t *out, void *stream);
int sw_launch_extend(const SwDev &D, const SwOptsDev &O, int grid_waves, int grid_pk, void *stream);
int sw_launch_global(const SwDev &D, const SwOptsDev &O, int grid_waves, int grid_pk, int grid_lds, int lds,
                     void *stream, void *ev_a, void *ev_b);
void sw_release(SwResident &r);

}  // namespace prgpu
