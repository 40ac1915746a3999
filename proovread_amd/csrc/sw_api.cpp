// Host side of the SW stage C-ABI (include/prgpu.h pr_sw_*).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/prgpu.h"
#include "aln_dev.h"
#include "sw_dev.h"
#include "sw_pk.h"
#include "xchg_dev.h"

using namespace prgpu;

// accessors defined in prgpu_api.cpp
SwResident &ctx_sw(pr_ctx *c);
void ctx_sw_batch_changed(pr_ctx *c);
hipStream_t ctx_stream(pr_ctx *c);
int ctx_device(pr_ctx *c);
int ctx_ncu(pr_ctx *c);
hipEvent_t ctx_event(pr_ctx *c, int i);
int pr_set_error(int code, const char *msg);

#define HIPCHK(x)                                                                 \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::string m_ = std::string(#x) + " failed: " + hipGetErrorString(e_); \
            return pr_set_error(PR_ERR_HIP, m_.c_str());                          \
        }                                                                         \
    } while (0)

enum SwBuf {
    SB_SR, SB_SR_OFF, SB_LR, SB_LR_OFF, SB_T_SR, SB_T_LR, SB_T_STRAND, SB_T_QBEG, SB_T_RBEG, SB_T_SLEN,
    SB_QB, SB_QE, SB_RB, SB_RE, SB_SCORE, SB_TRUESC, SB_W, SB_PASS, SB_GSCORE, SB_POS, SB_NCIG, SB_STATUS,
    SB_CIG, SB_Z
};
static const int SB_CELLS = 24;
// layout of the SB_CELLS buffer (zeroed per launch): [0,24) canonical DP cells, [24,56)
// packed CIGAR kernel phase cycles, [64,68) the LDS CIGAR kernel's dequeue counter
static const size_t CELLS_BYTES = 128;
static const size_t CELLS_WORK_OFF = 64;
static const int SB_PERM = 25;
static const int SB_BUCKET = 26;
static const int SB_X = 27;
static const int SB_XTRY = 28;
static const int SB_LIST = 29;
static const int SB_CIGSLOT = 30;   // int64 [n+1] prefix of the per-task CIGAR slots
static const int SB_CIGAT = 31;     // int64 [n] first op of each task's CIGAR
static const int SB_EHG = 32;       // HBM DP rows of the general CIGAR kernel (long queries)
static const int SB_CIGOFF = 33;    // pr_sw_download compaction: prefix of ncigar
static const int SB_CIGOUT = 34;    //                            compacted ops
static const size_t SPILL_OFF = 96;   // in the SB_CELLS buffer: 3 x u64 overflow counters
// bwa mode (aln_kernels.hip)
enum AlnBuf {
    SB_CHAIN = 35, SB_SEEDOFF, SB_SEL, SB_EXTF, SB_DEC, SB_RESUME, SB_ACNT, SB_AREG, SB_AIX, SB_PSCORE, SB_NPK,
    SB_FDONE, SB_PREQ, SB_NOUT, SB_OLIST, SB_OFLAG, SB_ATEMP, SB_AOFF, SB_ALIST, SB_AFLAG, SB_PPOOL, SB_GLIST,
    SB_GKEY0, SB_GKEY1, SB_GCNT, SB_GLROFF, SB_GPIPE, SB_GDOWN, SB_SCANIN, SB_TLIST, SB_CNEXT, SB_HPREV, SB_ABOX, SB_RSNAP, SB_KEYC, SB_NBUF
};
static_assert(SB_NBUF <= 80, "SwResident buffer table");

void prgpu_mem_note(const char *grp, int id, int64_t delta);
int prgpu_oom(const char *grp, int id, size_t want);

namespace prgpu {
void sw_release(SwResident &r) {
    for (void *&e : r.ext_ev.ev)
        if (e) (void)hipEventDestroy((hipEvent_t)e), e = nullptr;
    r.ext_ev.n = 0;
    if (r.side) (void)hipStreamDestroy((hipStream_t)r.side);
    for (void *&e : r.side_ev)
        if (e) (void)hipEventDestroy((hipEvent_t)e), e = nullptr;
    r.side = nullptr;
    for (int i = 0; i < 80; ++i) {
        if (r.buf[i]) (void)hipFree(r.buf[i]), prgpu_mem_note("sw", i, -(int64_t)r.cap[i]);
        r.buf[i] = nullptr;
        r.cap[i] = 0;
    }
    r.loaded = false;
}
}  // namespace prgpu


static int ensure(SwResident &r, int id, size_t bytes) {
    if (r.buf[id] && r.cap[id] >= bytes) return 0;
    if (r.buf[id]) (void)hipFree(r.buf[id]), prgpu_mem_note("sw", id, -(int64_t)r.cap[id]);
    r.buf[id] = nullptr;
    r.cap[id] = 0;
    const size_t want = bytes + 64;   // slack: kernels read whole dwords at the end of byte pools
    if (hipMalloc(&r.buf[id], want) != hipSuccess) {
        r.buf[id] = nullptr;
        return prgpu_oom("sw", id, want);
    }
    r.cap[id] = want;
    prgpu_mem_note("sw", id, (int64_t)want);
    return 0;
}
// The long-read pool starts SB_LR_FRONT bytes into its buffer: the extension kernels read
// 16-byte reference windows that may begin up to 15 bytes before a read (reverse strand).
static constexpr size_t SB_LR_FRONT = 64;
static uint8_t *lr_pool(SwResident &r) { return (uint8_t *)r.buf[SB_LR] + SB_LR_FRONT; }

template <class T>
static int up(SwResident &r, int id, const T *h, size_t n, hipStream_t s) {
    int rc = ensure(r, id, n * sizeof(T));
    if (rc) return rc;
    if (n && h) HIPCHK(hipMemcpyAsync(r.buf[id], h, n * sizeof(T), hipMemcpyHostToDevice, s));
    return 0;
}

extern "C" void pr_sw_opts_default(pr_sw_opts *o, int finish) {
    o->bin_size = 0;
    o->bin_length = 0.0;
    o->drop_ratio = finish ? 0.75 : 0.0;   // -D (proovread.cfg:325 / 332)
    o->mask_level = 0.5;
    o->mask_level_redun = 0.95;
    o->max_chain_gap = 10000;
    o->a = 5;
    o->pen_clip5 = o->pen_clip3 = 30;
    o->zdrop = 100;
    if (finish) {
        o->b = 13; o->o_del = 15; o->o_ins = 19; o->e_del = 3; o->e_ins = 3; o->w = 30;
        o->min_score_per_base = 4.0;
    } else {
        o->b = 11; o->o_del = 2; o->o_ins = 1; o->e_del = 4; o->e_ins = 3; o->w = 40;
        o->min_score_per_base = 2.5;
    }
}

// dev_tasks: bwa mode with the seeds already in HBM (the dense list of pr_seed_gpu_map, n_task
// of them, grouped by read; seed_off_h its per-read prefix on the host); b's task fields unused
// dev_sr / dev_lr (may be null): device copies of b's read pools (e.g. the seeding's), copied on
// the device instead of uploading b->sr_seq / b->lr_seq
static int sw_upload_impl(pr_ctx *c, const pr_sw_batch *b, const pr_seed_task *dev_tasks, const int64_t *seed_off_h,
                          const uint8_t *dev_sr = nullptr, const uint8_t *dev_lr = nullptr) {
    if (!c || !b) return pr_set_error(PR_ERR_ARG, "null arg");
    if (b->n_sr < 0 || b->n_lr < 0 || b->n_task < 0) return pr_set_error(PR_ERR_ARG, "negative sizes");
    HIPCHK(hipSetDevice(ctx_device(c)));
    SwResident &r = ctx_sw(c);
    hipStream_t s = ctx_stream(c);
    ctx_sw_batch_changed(c);   // an exchange of the previous batch must not be consumed
    int qmax = 1;
    for (int i = 0; i < b->n_sr; ++i) {
        const int64_t l = b->sr_off[i + 1] - b->sr_off[i];
        if (l < 0) return pr_set_error(PR_ERR_ARG, "sr_off not monotone");
        if (l > 1000) return pr_set_error(PR_ERR_ARG, "short read longer than 1000 (proovread:457 limit)");
        if (l > qmax) qmax = (int)l;
    }
    for (int i = 0; i < b->n_lr; ++i)
        if (b->lr_off[i + 1] < b->lr_off[i] || b->lr_off[i + 1] - b->lr_off[i] > (1 << 30))
            return pr_set_error(PR_ERR_ARG, "lr_off not monotone");
    for (int64_t t = 0; t < b->n_task && !dev_tasks; ++t) {
        const int sr = b->t_sr[t], lr = b->t_lr[t];
        if (sr < 0 || sr >= b->n_sr || lr < 0 || lr >= b->n_lr)
            return pr_set_error(PR_ERR_ARG, "task references a missing read");
        const int64_t lq = b->sr_off[sr + 1] - b->sr_off[sr], L = b->lr_off[lr + 1] - b->lr_off[lr];
        if (b->t_slen[t] <= 0 || b->t_qbeg[t] < 0 || b->t_qbeg[t] + b->t_slen[t] > lq || b->t_rbeg[t] < 0 ||
            b->t_rbeg[t] + b->t_slen[t] > L)
            return pr_set_error(PR_ERR_ARG, "seed outside its reads");
    }
    const int64_t nt = b->n_task;
    const bool bwa = b->t_chain != nullptr || dev_tasks;
    std::vector<int64_t> seed_off;
    if (dev_tasks) {
        seed_off.assign(seed_off_h, seed_off_h + b->n_sr + 1);
    } else if (bwa) {   // seeds grouped by short read, then chain
        if (nt >= (int64_t)1 << 31) return pr_set_error(PR_ERR_CAPACITY, "more than 2^31 seeds in one batch");
        seed_off.assign((size_t)b->n_sr + 1, 0);
        for (int64_t t = 0; t < nt; ++t) {
            if (t && (b->t_sr[t] < b->t_sr[t - 1] || (b->t_sr[t] == b->t_sr[t - 1] && b->t_chain[t] < b->t_chain[t - 1])))
                return pr_set_error(PR_ERR_ARG, "bwa mode: seeds must be grouped by short read, then chain");
            ++seed_off[(size_t)b->t_sr[t] + 1];
        }
        for (int i = 0; i < b->n_sr; ++i) seed_off[(size_t)i + 1] += seed_off[(size_t)i];
        r.n_rank0 = 0;
        for (int64_t t = 0; t < nt; ++t)
            r.n_rank0 += (t == 0 || b->t_sr[t] != b->t_sr[t - 1] || b->t_chain[t] != b->t_chain[t - 1]) ? 1 : 0;
    }
    r.n_big = 0;
    if (bwa)
        for (int i = 0; i < b->n_sr; ++i) r.n_big += seed_off[(size_t)i + 1] - seed_off[(size_t)i] > ALN_WAVE_SEEDS;
    int rc;
    if ((rc = up(r, SB_SR, dev_sr ? nullptr : b->sr_seq, (size_t)b->sr_off[b->n_sr], s)) ||
        (rc = up(r, SB_SR_OFF, b->sr_off, (size_t)b->n_sr + 1, s)) ||
        (rc = ensure(r, SB_LR, (size_t)b->lr_off[b->n_lr] + SB_LR_FRONT)) ||
        (rc = up(r, SB_LR_OFF, b->lr_off, (size_t)b->n_lr + 1, s)))
        return rc;
    if (!dev_lr && b->lr_off[b->n_lr])
        HIPCHK(hipMemcpyAsync(lr_pool(r), b->lr_seq, (size_t)b->lr_off[b->n_lr], hipMemcpyHostToDevice, s));
    if (dev_sr && b->sr_off[b->n_sr])
        HIPCHK(hipMemcpyAsync(r.buf[SB_SR], dev_sr, (size_t)b->sr_off[b->n_sr], hipMemcpyDeviceToDevice, s));
    if (dev_lr && b->lr_off[b->n_lr])
        HIPCHK(hipMemcpyAsync(lr_pool(r), dev_lr, (size_t)b->lr_off[b->n_lr], hipMemcpyDeviceToDevice, s));
    if (dev_tasks) {   // unpack the device seed list into the task columns, count the first seeds
        if ((rc = ensure(r, SB_T_SR, (size_t)nt * 4)) || (rc = ensure(r, SB_T_LR, (size_t)nt * 4)) ||
            (rc = ensure(r, SB_T_STRAND, (size_t)nt)) || (rc = ensure(r, SB_T_QBEG, (size_t)nt * 4)) ||
            (rc = ensure(r, SB_T_RBEG, (size_t)nt * 4)) || (rc = ensure(r, SB_T_SLEN, (size_t)nt * 4)) ||
            (rc = ensure(r, SB_CHAIN, (size_t)nt * 4)) || (rc = ensure(r, SB_ACNT, 64)) ||
            (rc = ensure(r, SB_CNEXT, ((size_t)nt + 1) * 4)))
            return rc;
        HIPCHK(hipMemsetAsync(r.buf[SB_ACNT], 0, 64, s));
        int e = aln_launch_unpack_seeds(dev_tasks, nt, (int32_t *)r.buf[SB_T_SR], (int32_t *)r.buf[SB_T_LR],
                                        (uint8_t *)r.buf[SB_T_STRAND], (int32_t *)r.buf[SB_T_QBEG],
                                        (int32_t *)r.buf[SB_T_RBEG], (int32_t *)r.buf[SB_T_SLEN],
                                        (int32_t *)r.buf[SB_CHAIN], (int32_t *)r.buf[SB_ACNT],
                                        (int32_t *)r.buf[SB_CNEXT], (void *)s);
        if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        int32_t n0 = 0;
        HIPCHK(hipMemcpyAsync(&n0, r.buf[SB_ACNT], 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        r.n_rank0 = n0;
        r.cnext_ready = true;
    } else if ((rc = up(r, SB_T_SR, b->t_sr, nt, s)) || (rc = up(r, SB_T_LR, b->t_lr, nt, s)) ||
               (rc = up(r, SB_T_STRAND, b->t_strand, nt, s)) || (rc = up(r, SB_T_QBEG, b->t_qbeg, nt, s)) ||
               (rc = up(r, SB_T_RBEG, b->t_rbeg, nt, s)) || (rc = up(r, SB_T_SLEN, b->t_slen, nt, s))) {
        return rc;
    }
    const size_t n4 = (size_t)(nt + 1) * 4;
    for (int id : {SB_QB, SB_QE, SB_RB, SB_RE, SB_SCORE, SB_TRUESC, SB_W, SB_GSCORE, SB_POS, SB_NCIG, SB_STATUS})
        if ((rc = ensure(r, id, n4))) return rc;
    if ((rc = ensure(r, SB_PERM, (size_t)(nt + 1) * 4)) || (rc = ensure(r, SB_KEYC, (size_t)(nt + 1) * 4)) || (rc = ensure(r, SB_BUCKET, (SW_NBUCKET + 16 + PK_SCAN + 1) * 4)) ||
        (rc = ensure(r, SB_X, (size_t)(nt + 1) * 4 * 12)) || (rc = ensure(r, SB_XTRY, (size_t)nt + 1)) ||
        (rc = ensure(r, SB_LIST, (size_t)(nt + 1 + (int64_t)PK_NB * PK_SEG) * 4)))
        return rc;
    r.bwa = bwa;
    if (!dev_tasks) r.cnext_ready = false;
    r.read_id0 = b->read_id0;
    r.n_aln = 0;
    if (bwa) {
        const size_t n1 = (size_t)nt + 1, r1 = (size_t)b->n_sr + 1;
        if ((!dev_tasks && (rc = up(r, SB_CHAIN, b->t_chain, (size_t)nt, s))) ||
            (rc = up(r, SB_SEEDOFF, seed_off.data(), r1, s)) ||
            (rc = ensure(r, SB_SEL, n1)) || (rc = ensure(r, SB_EXTF, n1)) || (rc = ensure(r, SB_DEC, n1)) ||
            (rc = ensure(r, SB_RESUME, r1 * 4)) || (rc = ensure(r, SB_ACNT, 64)) ||
            (rc = ensure(r, SB_AREG, n1 * sizeof(AlnReg))) || (rc = ensure(r, SB_AIX, n1 * 4)) ||
            (rc = ensure(r, SB_PSCORE, n1 * 4)) || (rc = ensure(r, SB_NPK, r1 * 4)) || (rc = ensure(r, SB_FDONE, r1)) ||
            (rc = ensure(r, SB_NOUT, r1 * 4)) || (rc = ensure(r, SB_OLIST, n1 * 4)) || (rc = ensure(r, SB_OFLAG, n1 * 4)) ||
            (rc = ensure(r, SB_AOFF, r1 * 8)) || (rc = ensure(r, SB_ALIST, n1 * 4)) || (rc = ensure(r, SB_AFLAG, n1 * 4)) ||
            (rc = ensure(r, SB_PREQ, 1024 * sizeof(AlnPatch))) || (rc = ensure(r, SB_CIGSLOT, n1 * 8)) ||
            (rc = ensure(r, SB_TLIST, n1 * 4)) || (rc = ensure(r, SB_CNEXT, n1 * 4)) || (rc = ensure(r, SB_HPREV, n1 * 4)) ||
            (rc = ensure(r, SB_ABOX, n1 * sizeof(AlnBox))) || (rc = ensure(r, SB_RSNAP, r1 * 4)) ||
            (rc = ensure(r, SB_CIGAT, n1 * 8)) || (rc = ensure(r, SB_PASS, n1)) || (rc = ensure(r, SB_CELLS, CELLS_BYTES)))
            return rc;
        size_t tb = aln_scan_temp_bytes(nt);
        tb = std::max(tb, aln_scan_temp_bytes(b->n_sr));
        tb = std::max(tb, aln_group_temp_bytes(nt, b->n_lr));
        if ((rc = ensure(r, SB_ATEMP, tb))) return rc;
        r.cig_slots = 0;
        HIPCHK(hipStreamSynchronize(s));
        r.loaded = true;
        r.n_task = nt;
        r.n_sr = b->n_sr;
        r.n_lr = b->n_lr;
        r.qmax = qmax;
        return 0;
    }
    // CIGAR slots sized from the short-read lengths, plus a spill reserve for overflows
    // (PRGPU_SW_CIG_SLOT: a fixed slot size, a test hook that sends CIGARs to the overflow pass)
    std::vector<int64_t> slot((size_t)nt + 1, 0);
    const int forced = getenv("PRGPU_SW_CIG_SLOT") ? atoi(getenv("PRGPU_SW_CIG_SLOT")) : 0;
    for (int64_t t = 0; t < nt; ++t) {
        const int sr = b->t_sr[t];
        const int cs = forced > 0 ? forced : cig_slot_ops((int)(b->sr_off[sr + 1] - b->sr_off[sr]));
        slot[(size_t)t + 1] = slot[(size_t)t] + cs;
    }
    const int64_t slots = slot[(size_t)nt];
    const int64_t reserve = slots / 16 > (1 << 20) ? slots / 16 : (1 << 20);
    if ((rc = ensure(r, SB_PASS, (size_t)nt + 1)) || (rc = ensure(r, SB_CIG, (size_t)(slots + reserve) * 4)) ||
        (rc = up(r, SB_CIGSLOT, slot.data(), slot.size(), s)) || (rc = ensure(r, SB_CIGAT, (size_t)(nt + 1) * 8)) ||
        (rc = ensure(r, SB_CELLS, CELLS_BYTES)))
        return rc;
    r.cig_slots = slots;
    HIPCHK(hipStreamSynchronize(s));
    r.loaded = true;
    r.n_task = nt;
    r.n_sr = b->n_sr;
    r.n_lr = b->n_lr;
    r.qmax = qmax;
    return 0;
}

extern "C" int pr_sw_upload(pr_ctx *c, const pr_sw_batch *b) { return sw_upload_impl(c, b, nullptr, nullptr); }

// the iteration's SW upload with the device-resident seeds of pr_seed_gpu_map (prgpu_api.cpp)
int sw_upload_device_seeds(pr_ctx *c, const pr_sw_batch *b, const pr_seed_task *dev_tasks, const int64_t *seed_off_h,
                           const uint8_t *dev_sr, const uint8_t *dev_lr) {
    return sw_upload_impl(c, b, dev_tasks, seed_off_h, dev_sr, dev_lr);
}

static AlnDev aln_dev(SwResident &r, const SwDev &D, const pr_sw_opts *o) {
    AlnDev A;
    std::memset(&A, 0, sizeof A);
    A.n_task = r.n_task;
    A.n_sr = (int32_t)r.n_sr;
    A.n_lr = (int32_t)r.n_lr;
    A.read_id0 = r.read_id0;
    A.n_big = r.n_big;
    A.seed_off = (const int64_t *)r.buf[SB_SEEDOFF];
    A.t_sr = D.t_sr;
    A.t_lr = D.t_lr;
    A.t_qbeg = D.t_qbeg;
    A.t_rbeg = D.t_rbeg;
    A.t_slen = D.t_slen;
    A.t_chain = (const int32_t *)r.buf[SB_CHAIN];
    A.t_strand = D.t_strand;
    A.sr_off = D.sr_off;
    A.lr_off = D.lr_off;
    A.sr = D.sr;
    A.lr = D.lr;
    A.o_qb = D.o_qb; A.o_qe = D.o_qe; A.o_rb = D.o_rb; A.o_re = D.o_re;
    A.o_score = D.o_score; A.o_truesc = D.o_truesc; A.o_w = D.o_w;
    A.o_pass = D.o_pass;
    A.sel = (uint8_t *)r.buf[SB_SEL];
    A.ext = (uint8_t *)r.buf[SB_EXTF];
    A.dec = (uint8_t *)r.buf[SB_DEC];
    A.resume = (int32_t *)r.buf[SB_RESUME];
    A.counter = (int32_t *)r.buf[SB_ACNT];
    A.tlist = (int32_t *)r.buf[SB_TLIST];
    A.cnext = (int32_t *)r.buf[SB_CNEXT];
    A.cnext_ready = r.cnext_ready ? 1 : 0;
    A.hprev = getenv("PRGPU_ALN_NO_HPREV") ? nullptr : (int32_t *)r.buf[SB_HPREV];
    A.box = (AlnBox *)r.buf[SB_ABOX];
    A.R = (AlnReg *)r.buf[SB_AREG];
    A.ix = (int32_t *)r.buf[SB_AIX];
    A.pscore = (int32_t *)r.buf[SB_PSCORE];
    A.npk = (int32_t *)r.buf[SB_NPK];
    A.fdone = (uint8_t *)r.buf[SB_FDONE];
    A.preq = (AlnPatch *)r.buf[SB_PREQ];
    A.preq_cap = (int32_t)(r.cap[SB_PREQ] / sizeof(AlnPatch));
    A.nout = (int32_t *)r.buf[SB_NOUT];
    A.olist = (int32_t *)r.buf[SB_OLIST];
    A.oflag = (int32_t *)r.buf[SB_OFLAG];
    A.a = o->a; A.b = o->b; A.o_del = o->o_del; A.e_del = o->e_del; A.o_ins = o->o_ins; A.e_ins = o->e_ins;
    A.w = o->w;
    A.max_chain_gap = o->max_chain_gap;
    A.min_score_per_base = o->min_score_per_base;
    A.drop_ratio = o->drop_ratio;
    A.mask_level = o->mask_level;
    A.mask_level_redun = o->mask_level_redun;
    return A;
}

// direction slabs of the band-80 ring kernel when it runs beside the fused packed CIGAR kernel
// (sw_launch_global's side path): after the packed kernel's slabs in SB_Z; null when SB_Z has no
// room for both (split packed kernel, or PRGPU_RING80_SIDE=0)
static void *ring_side_z(const SwResident &r, const SwDev &D, int grid_pk, int grid_w) {
    const char *e = getenv("PRGPU_RING80_SIDE");
    if ((e && e[0] == '0') || D.pk_chunk > 0) return nullptr;
    const size_t pk = ((size_t)D.z_pk_slab * sizeof(PkDir) * grid_pk + 255) & ~(size_t)255;
    const size_t ring = (size_t)D.z_ring_slab * 4 * grid_w;
    if (!r.buf[SB_Z] || r.cap[SB_Z] < pk + ring) return nullptr;
    return (uint8_t *)r.buf[SB_Z] + pk;
}

// the side stream (and its events) of the bwa-mode rounds
static int side_stream(SwResident &r) {
    if (r.side) return 0;
    hipStream_t st;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    r.side = (void *)st;
    for (void *&ev : r.side_ev) {
        hipEvent_t x;
        HIPCHK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
        ev = (void *)x;
    }
    return 0;
}

// The packed CIGAR pass's task order (sorted by key, padded to 128-task segments), then its
// launch geometry.  Default: the fused kernel (DP and backtrack per segment in one wave, a
// slab per resident wave).  PRGPU_PK_SPLIT=1: the segment count read back, split into chunks
// whose slabs (one per segment, PK_TMAX rows) fit PRGPU_PK_SLAB_GB (default 4 GB, at most half
// of the free device memory), each chunk
// a DP launch and a backtrack launch (measured at configs[1]: DP 43.4 + backtrack 15.4 ms
// against 58.8 ms fused -- the walk is latency- and issue-bound).
static int pk_prepare(pr_ctx *c, SwResident &r, SwDev &D, const SwOptsDev &O) {
    D.pk_chunk = 0;
    const char *fw = getenv("PRGPU_PK_WIN");
    // the fused kernel's backtrack window: 8 rows (no scratch, ~3 k fewer unrolled instructions;
    // 55.9 against 56.2 ms with 16 after the branch-free step), PRGPU_PK_WIN=16 for 16
    D.pk_bt_win = fw && atoi(fw) == 16 ? 16 : 8;
    if (!O.pk) return 0;
    hipStream_t s = ctx_stream(c);
    int e = sw_launch_pk_order(D, O, 0, (void *)s);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    const char *sp = getenv("PRGPU_PK_SPLIT");
    if (!sp || !atoi(sp)) return 0;
    int32_t len = 0;
    HIPCHK(hipMemcpyAsync(&len, D.pk_bucket + PK_SCAN, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const int64_t nseg = len / PK_SEG;
    const size_t slab = (size_t)D.z_pk_slab * sizeof(PkDir);
    const char *gb = getenv("PRGPU_PK_SLAB_GB");
    double budget = (gb ? atof(gb) : 4.0) * (double)(1ull << 30);
    size_t free_b = 0, total_b = 0;   // never more than half of what is free
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && budget > 0.5 * (double)free_b) budget = 0.5 * (double)free_b;
    int64_t per = (int64_t)(budget / (double)slab);
    per = per < 64 ? 64 : per;
    const int64_t nch = nseg > 0 ? (nseg + per - 1) / per : 1;
    const int64_t chunk = nseg > 0 ? (nseg + nch - 1) / nch : 1;
    if ((size_t)chunk * slab > r.cap[SB_Z]) {
        int rc = ensure(r, SB_Z, (size_t)chunk * slab);
        if (rc) return rc;
    }
    D.z = (uint8_t *)r.buf[SB_Z];
    D.pk_chunk = (int)chunk;
    D.pk_nseg_bound = nseg;
    const char *bw = getenv("PRGPU_PK_BT_WIN");
    D.pk_bt_win = bw && (atoi(bw) == 16 || atoi(bw) == 4) ? atoi(bw) : 8;
    D.pk_bt_grid = ctx_ncu(c) * sw_pk_bt_occupancy(D.pk_bt_win);
    return 0;
}

// bwa mode: extension rounds (mem_chain2aln), the final pass (mem_sort_dedup_patch ..
// mem_reg2sam) with mem_patch_reg rounds, then the CIGAR pass over the reported alignments
static int bwa_launch(pr_ctx *c, SwResident &r, SwDev &D, const SwOptsDev &O, const pr_sw_opts *o, int grid_w,
                      int grid_pk, int grid_g, int lds_glob) {
    hipStream_t s = ctx_stream(c);
    int rc, e;
    D.sel = (const uint8_t *)r.buf[SB_SEL];
    AlnDev A = aln_dev(r, D, o);
    r.ext_rounds = 0;
    r.n_ext = r.n_rank0;   // rank-0 seeds, extended in the first round
    r.n_patch = 0;
    r.n_aln = 0;
    HIPCHK(hipEventRecord(ctx_event(c, 2), s));
    if (!r.bt_ev[0])
        for (void *&ev : r.bt_ev) {
            hipEvent_t x;
            HIPCHK(hipEventCreate(&x));
            ev = (void *)x;
        }
    hipEvent_t *bt = reinterpret_cast<hipEvent_t *>(r.bt_ev);
    r.ms_walk = r.ms_final = r.ms_final_early = 0.f;
    auto bt_add = [&](float &acc, int k) {   // (after a sync that follows event bt[k + 1])
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, bt[k], bt[k + 1]) == hipSuccess) acc += ms;
        (void)hipGetLastError();
    };
    HIPCHK(hipMemsetAsync(A.counter, 0, 16, s));
    if ((e = aln_launch_init(A, (void *)s))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    if ((e = aln_launch_list(A, (void *)s))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    // the chain-head links only feed the walk: built on the side stream beside round 0's extension
    bool heads_side = false;
    if (A.hprev) {
        if ((rc = side_stream(r))) return rc;
        HIPCHK(hipEventRecord((hipEvent_t)r.side_ev[0], s));
        HIPCHK(hipStreamWaitEvent((hipStream_t)r.side, (hipEvent_t)r.side_ev[0], 0));
        if ((e = aln_launch_heads(A, r.side))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        HIPCHK(hipEventRecord((hipEvent_t)r.side_ev[2], (hipStream_t)r.side));
        heads_side = true;
    }
    int32_t cnt[4] = {0, 0, 0, 0};
    int64_t n_list = r.n_rank0;   // round 0: every chain's first seed (listed after the init kernel)
    D.tsel = A.tlist;
    bool early = false;
    for (;;) {   // mem_chain2aln: every round extends the listed seeds, the walk resumes
        D.tsel_n = n_list;
        HIPCHK(hipMemsetAsync(A.counter, 0, 8, s));
        if (n_list) {
            e = sw_launch_extend(D, O, ctx_ncu(c) * 16, grid_pk, (void *)s, &r.ext_ev);
            if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        }
        if (heads_side) {
            HIPCHK(hipStreamWaitEvent(s, (hipEvent_t)r.side_ev[2], 0));
            heads_side = false;
        }
        HIPCHK(hipEventRecord(bt[0], s));
        if ((e = aln_launch_walk(A, (void *)s))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        HIPCHK(hipEventRecord(bt[1], s));
        if ((e = aln_launch_list(A, (void *)s))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        HIPCHK(hipMemcpyAsync(cnt, A.counter, 16, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        bt_add(r.ms_walk, 0);
        ++r.ext_rounds;
        r.n_ext += cnt[0];
        // after the first resumed walk most reads are decided: their final pass runs on a side
        // stream while the later (small, latency-bound) rounds finish the rest; the late pass
        // below skips them (fdone) and also replays any read whose patch score the early pass
        // would have had to request
        if (r.ext_rounds == 1 && cnt[0] > 0 && !getenv("PRGPU_BWA_NO_EARLY_FINAL")) {
            if ((rc = side_stream(r))) return rc;
            // the reads finished now, snapshotted on the main stream: the early pass never reads
            // the live resume array the later rounds' walks write
            int32_t *snap = (int32_t *)r.buf[SB_RSNAP];
            HIPCHK(hipMemcpyAsync(snap, A.resume, (size_t)r.n_sr * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipEventRecord((hipEvent_t)r.side_ev[0], s));
            HIPCHK(hipStreamWaitEvent((hipStream_t)r.side, (hipEvent_t)r.side_ev[0], 0));
            HIPCHK(hipEventRecord(bt[4], (hipStream_t)r.side));
            if ((e = aln_launch_final(A, r.side, snap))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
            HIPCHK(hipEventRecord(bt[5], (hipStream_t)r.side));
            HIPCHK(hipEventRecord((hipEvent_t)r.side_ev[1], (hipStream_t)r.side));
            early = true;
        }
        if (getenv("PRGPU_BWA_DEBUG")) fprintf(stderr, "[bwa] round %d: %d requests\n", r.ext_rounds, cnt[0]);
        if (cnt[0] == 0) break;
        if (r.ext_rounds > r.n_task + 2) return pr_set_error(PR_ERR_HIP, "bwa mode: extension rounds do not converge");
        n_list = cnt[0];
    }
    D.tsel = nullptr;
    bool comp_timed = false;
    if (early) {   // the reads the early pass skips, beside it (disjoint reads), then join it
        HIPCHK(hipEventRecord(bt[6], s));
        if (!getenv("PRGPU_BWA_NO_COMPLEMENT") &&
            (e = aln_launch_final(A, (void *)s, (const int32_t *)r.buf[SB_RSNAP], true)))
            return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        HIPCHK(hipEventRecord(bt[7], s));
        HIPCHK(hipStreamWaitEvent(s, (hipEvent_t)r.side_ev[1], 0));
        comp_timed = true;
    }
    for (int round = 0;; ++round) {   // final pass; mem_patch_reg global scores in extra rounds
        HIPCHK(hipMemsetAsync(A.counter, 0, 16, s));
        HIPCHK(hipEventRecord(bt[2], s));
        if ((e = aln_launch_final(A, (void *)s, nullptr))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        HIPCHK(hipEventRecord(bt[3], s));
        HIPCHK(hipMemcpyAsync(cnt, A.counter, 16, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        bt_add(r.ms_final, 2);
        if (comp_timed) {   // (the side stream joined before this sync)
            bt_add(r.ms_final, 6);
            bt_add(r.ms_final_early, 4);
            comp_timed = false;
        }
        if (getenv("PRGPU_BWA_DEBUG")) fprintf(stderr, "[bwa] final round %d: %d patch requests\n", round, cnt[1]);
        if (cnt[1] == 0) break;
        if (round > r.n_task + 2) return pr_set_error(PR_ERR_HIP, "bwa mode: patch rounds do not converge");
        const int n_req = cnt[1] < A.preq_cap ? cnt[1] : A.preq_cap;
        const int64_t stride = 2 * ((int64_t)r.qmax + 2);
        if ((rc = ensure(r, SB_PPOOL, (size_t)n_req * (size_t)stride * 4))) return rc;
        if ((e = aln_launch_patch(A, n_req, (int32_t *)r.buf[SB_PPOOL], stride, (void *)s)))
            return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        r.n_patch += n_req;
        if (cnt[1] > A.preq_cap) {   // requests beyond the list are made again next round
            HIPCHK(hipStreamSynchronize(s));
            if ((rc = ensure(r, SB_PREQ, (size_t)cnt[1] * sizeof(AlnPatch)))) return rc;
            A.preq = (AlnPatch *)r.buf[SB_PREQ];
            A.preq_cap = (int32_t)(r.cap[SB_PREQ] / sizeof(AlnPatch));
        }
    }
    // CIGAR slots of the reported alignments, the pool, then the CIGAR pass over them
    {
        const int64_t nmax = (r.n_task > r.n_sr ? r.n_task : r.n_sr) + 1;
        if ((rc = ensure(r, SB_SCANIN, (size_t)nmax * 8))) return rc;
    }
    if (getenv("PRGPU_BWA_DEBUG"))
        fprintf(stderr, "[bwa] rounds %d, extended %lld, patches %lld\n", r.ext_rounds, (long long)r.n_ext,
                (long long)r.n_patch);
    if ((e = aln_launch_cig_slots(A, (int64_t *)r.buf[SB_CIGSLOT], (int64_t *)r.buf[SB_SCANIN], r.buf[SB_ATEMP],
                                  r.cap[SB_ATEMP], (void *)s)))
        return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    int64_t slots = 0;
    HIPCHK(hipMemcpyAsync(&slots, (int64_t *)r.buf[SB_CIGSLOT] + r.n_task, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const int64_t reserve = slots / 16 > (1 << 20) ? slots / 16 : (1 << 20);
    if ((rc = ensure(r, SB_CIG, (size_t)(slots + reserve) * 4))) return rc;
    r.cig_slots = slots;
    D.o_cig = (uint32_t *)r.buf[SB_CIG];
    D.cig_slot = (const int64_t *)r.buf[SB_CIGSLOT];
    D.spill_base = slots;
    if (r.n_task) HIPCHK(hipMemcpyAsync(r.buf[SB_CIGAT], r.buf[SB_CIGSLOT], (size_t)r.n_task * 8, hipMemcpyDeviceToDevice, s));
    if ((e = aln_launch_compact(A, (int64_t *)r.buf[SB_AOFF], (int64_t *)r.buf[SB_SCANIN], (int32_t *)r.buf[SB_ALIST],
                                (int32_t *)r.buf[SB_AFLAG], r.buf[SB_ATEMP], r.cap[SB_ATEMP], (void *)s)))
        return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    HIPCHK(hipMemcpyAsync(&r.n_aln, (int64_t *)r.buf[SB_AOFF] + r.n_sr, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    D.tsel = (const int32_t *)r.buf[SB_ALIST];   // the CIGAR pass over the reported alignments
    D.tsel_n = r.n_aln;
    HIPCHK(hipEventRecord(ctx_event(c, 3), s));
    if (r.n_aln) {
        if ((rc = pk_prepare(c, r, D, O))) return rc;
        if ((rc = side_stream(r))) return rc;
        e = sw_launch_global(D, O, grid_w, grid_pk, grid_g, lds_glob, (void *)s, (void *)ctx_event(c, 6),
                             (void *)ctx_event(c, 7), true, r.side, r.side_ev[0], r.side_ev[2],
                             ring_side_z(r, D, grid_pk, grid_w), r.side_ev[1]);
        if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    }
    unsigned long long sp[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(sp, D.spill, sizeof sp, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (sp[0]) {
        const size_t need = (size_t)(r.cig_slots + (int64_t)sp[1]) * 4;
        if (need > r.cap[SB_CIG]) {   // grow the pool, keeping the slots
            void *np = nullptr;
            if (hipMalloc(&np, need + need / 8) != hipSuccess) return prgpu_oom("sw CIGAR spill", SB_CIG, need + need / 8);
            HIPCHK(hipMemcpyAsync(np, r.buf[SB_CIG], (size_t)r.cig_slots * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
            (void)hipFree(r.buf[SB_CIG]);
            prgpu_mem_note("sw", SB_CIG, (int64_t)(need + need / 8) - (int64_t)r.cap[SB_CIG]);
            r.buf[SB_CIG] = np;
            r.cap[SB_CIG] = need + need / 8;
            D.o_cig = (uint32_t *)np;
        }
        HIPCHK(hipMemsetAsync(D.work, 0, 4, s));
        e = sw_launch_overflow(D, O, grid_g, lds_glob, (void *)s);
        if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    }
    r.n_overflow = (int64_t)sp[0];
    HIPCHK(hipEventRecord(ctx_event(c, 0), s));
    return 0;
}

extern "C" int pr_sw_launch(pr_ctx *c, const pr_sw_opts *o) {
    if (!c || !o) return pr_set_error(PR_ERR_ARG, "null arg");
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch (pr_sw_upload first)");
    if (o->a <= 0 || o->b < 0 || o->e_del <= 0 || o->e_ins <= 0 || o->w <= 0)
        return pr_set_error(PR_ERR_ARG, "bad scoring options");
    if ((long)o->a * r.qmax >= 8192)
        return pr_set_error(PR_ERR_ARG, "a * max read length must stay below 8192 (13-bit DP words)");
    if (o->w > 1000) return pr_set_error(PR_ERR_UNSUPPORTED, "band width w > 1000");
    if (o->a > 15 || o->b > 16) return pr_set_error(PR_ERR_UNSUPPORTED, "match score > 15 or mismatch penalty > 16");
    HIPCHK(hipSetDevice(ctx_device(c)));
    (void)hipGetLastError();   // a failed earlier call must not poison this one
    hipStream_t s = ctx_stream(c);
    SwOptsDev O;
    O.a = o->a; O.b = o->b; O.o_del = o->o_del; O.e_del = o->e_del; O.o_ins = o->o_ins; O.e_ins = o->e_ins;
    O.w = o->w; O.pen_clip5 = o->pen_clip5; O.pen_clip3 = o->pen_clip3; O.zdrop = o->zdrop;
    O.min_score_per_base = o->min_score_per_base;
    // the packed kernel's int16 frame holds |values| < 9000 for these penalties (sw_pk.h)
    O.pk = (o->o_del <= 32 && o->o_ins <= 32 && o->e_del <= 32 && o->e_ins <= 32 && !getenv("PRGPU_SW_NOPK")) ? 1 : 0;
    O.debug = getenv("PRGPU_SW_DEBUG") ? atoi(getenv("PRGPU_SW_DEBUG")) : 0;
    SwDev D;
    std::memset(&D, 0, sizeof D);
    D.n_task = r.n_task;
    D.qmax = r.qmax;
    // reference rows of a region: query + 2 x 2w of extension; a patched (merged) region of bwa
    // mode adds up to 4w more (mem_patch_reg's band bound)
    D.tmax = r.qmax + (r.bwa ? 8 : 4) * o->w + 8;
    D.sr = (const uint8_t *)r.buf[SB_SR];
    D.sr_off = (const int64_t *)r.buf[SB_SR_OFF];
    D.lr = lr_pool(r);
    D.lr_off = (const int64_t *)r.buf[SB_LR_OFF];
    D.t_sr = (const int32_t *)r.buf[SB_T_SR];
    D.t_lr = (const int32_t *)r.buf[SB_T_LR];
    D.t_strand = (const uint8_t *)r.buf[SB_T_STRAND];
    D.t_qbeg = (const int32_t *)r.buf[SB_T_QBEG];
    D.t_rbeg = (const int32_t *)r.buf[SB_T_RBEG];
    D.t_slen = (const int32_t *)r.buf[SB_T_SLEN];
    D.o_qb = (int32_t *)r.buf[SB_QB];
    D.o_qe = (int32_t *)r.buf[SB_QE];
    D.o_rb = (int32_t *)r.buf[SB_RB];
    D.o_re = (int32_t *)r.buf[SB_RE];
    D.o_score = (int32_t *)r.buf[SB_SCORE];
    D.o_truesc = (int32_t *)r.buf[SB_TRUESC];
    D.o_w = (int32_t *)r.buf[SB_W];
    D.o_pass = (uint8_t *)r.buf[SB_PASS];
    D.o_gscore = (int32_t *)r.buf[SB_GSCORE];
    D.o_pos = (int32_t *)r.buf[SB_POS];
    D.o_ncig = (int32_t *)r.buf[SB_NCIG];
    D.o_status = (int32_t *)r.buf[SB_STATUS];
    D.o_cig = (uint32_t *)r.buf[SB_CIG];
    D.cig_slot = (const int64_t *)r.buf[SB_CIGSLOT];
    D.o_cig_at = (int64_t *)r.buf[SB_CIGAT];
    D.spill = (unsigned long long *)((char *)r.buf[SB_CELLS] + SPILL_OFF);
    D.spill_base = r.cig_slots;
    D.cells = (unsigned long long *)r.buf[SB_CELLS];
    D.work = (int32_t *)((char *)r.buf[SB_CELLS] + CELLS_WORK_OFF);
    D.perm = (int32_t *)r.buf[SB_PERM];
    D.keyc = (int32_t *)r.buf[SB_KEYC];
    D.bucket = (int32_t *)r.buf[SB_BUCKET];
    D.x = (int32_t *)r.buf[SB_X];
    D.x_try = (uint8_t *)r.buf[SB_XTRY];
    D.list = (int32_t *)r.buf[SB_LIST];
    D.list_n = D.bucket + SW_NBUCKET;
    int rc0 = 0;
    D.pk_bucket = D.bucket + SW_NBUCKET + 16;
    // row of the general CIGAR kernel: (qmax+1) H/E words per lane + lane-major query bytes,
    // in LDS when it fits next to the kernel's static LDS, else in HBM (queries > ~500 bp)
    const int lds_ext = (r.qmax + 1) * SW_WAVE * 4;
    const int qpad = (r.qmax + 8) & ~3;
    const int lds_glob = lds_ext + SW_WAVE * qpad;
    const bool eh_hbm_g = lds_glob + 256 > 160 * 1024;
    // the wide-band extension kernel (tries with w > 80) keeps (qmax+2) words per lane
    const int lds_wide = (r.qmax + 2) * SW_WAVE * 4;
    const bool eh_hbm_x = (o->w << 1) > 80 && lds_wide + 256 > 160 * 1024;
    const bool eh_hbm = eh_hbm_g || eh_hbm_x;
    const int blocks_per_cu = eh_hbm ? 2 : ((160 * 1024) / (lds_glob + 64) > 0 ? (160 * 1024) / (lds_glob + 64) : 1);
    int grid_g = ctx_ncu(c) * (blocks_per_cu < 8 ? blocks_per_cu : 8);
    D.z_slab = (int64_t)D.tmax * ((r.qmax + 3) / 4) * 4 * SW_WAVE;
    {   // direction slabs of the general kernel within 4 GB
        const int64_t gmax = ((int64_t)4 << 30) / (D.z_slab > 0 ? D.z_slab : 1);
        if (grid_g > gmax) grid_g = (int)(gmax > 16 ? gmax : 16);
    }
    if (eh_hbm) {
        const int row = lds_glob > lds_wide ? lds_glob : lds_wide;
        D.eh_g_stride = (int64_t)((row + 255) & ~255) / 4;
        D.eh_g_blocks = grid_g;
        if ((rc0 = ensure(r, SB_EHG, (size_t)D.eh_g_stride * 4 * (size_t)grid_g))) return rc0;
        D.eh_g = (uint32_t *)r.buf[SB_EHG];
    }
    const int grid_w = ctx_ncu(c) * 12;                       // ring kernels: 3 waves per SIMD
    D.z_ring_slab = (int64_t)D.tmax * ((2 * 80 + 2 + 7) / 8) * SW_WAVE;
    const int grid_pk = ctx_ncu(c) * 8;                       // packed kernel: ~200 VGPRs, 2 waves per SIMD
    D.z_pk_slab = (int64_t)PK_TMAX * pk_npair(40) * SW_WAVE;
    size_t zb = (size_t)D.z_slab * grid_g > (size_t)D.z_ring_slab * 4 * grid_w
                    ? (size_t)D.z_slab * grid_g : (size_t)D.z_ring_slab * 4 * grid_w;
    if ((size_t)D.z_pk_slab * sizeof(PkDir) * grid_pk > zb) zb = (size_t)D.z_pk_slab * sizeof(PkDir) * grid_pk;
    if (O.pk) {   // the band-80 ring kernel's slabs after the packed kernel's (run beside it, ring_side_z)
        const size_t both = (((size_t)D.z_pk_slab * sizeof(PkDir) * grid_pk + 255) & ~(size_t)255) +
                            (size_t)D.z_ring_slab * 4 * grid_w;
        if (both > zb) zb = both;
    }
    int rc;
    if ((rc = ensure(r, SB_Z, zb))) return rc;
    D.z = (uint8_t *)r.buf[SB_Z];
    HIPCHK(hipMemsetAsync(r.buf[SB_CELLS], 0, CELLS_BYTES, s));
    for (void *&ev : r.ext_ev.ev)
        if (!ev) {
            hipEvent_t x;
            HIPCHK(hipEventCreate(&x));
            ev = (void *)x;
        }
    r.ext_ev.n = 0;
    r.ext_ev.dropped = 0;
    if (r.bwa) return bwa_launch(c, r, D, O, o, grid_w, grid_pk, grid_g, lds_glob);
    if (r.n_task == 0) return 0;
    HIPCHK(hipMemcpyAsync(r.buf[SB_CIGAT], r.buf[SB_CIGSLOT], (size_t)r.n_task * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipEventRecord(ctx_event(c, 2), s));
    int e = sw_launch_extend(D, O, ctx_ncu(c) * 16, grid_pk, (void *)s, &r.ext_ev);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));

    HIPCHK(hipEventRecord(ctx_event(c, 3), s));
    if ((rc = pk_prepare(c, r, D, O))) return rc;
    if ((rc = side_stream(r))) return rc;
    e = sw_launch_global(D, O, grid_w, grid_pk, grid_g, lds_glob, (void *)s, (void *)ctx_event(c, 6), (void *)ctx_event(c, 7),
                         true, r.side, r.side_ev[0], r.side_ev[2], ring_side_z(r, D, grid_pk, grid_w), r.side_ev[1]);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    // CIGARs longer than their slots: recompute those tasks into the spill area
    unsigned long long sp[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(sp, D.spill, sizeof sp, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (sp[0]) {
        const size_t need = (size_t)(r.cig_slots + (int64_t)sp[1]) * 4;
        if (need > r.cap[SB_CIG]) {   // grow the pool, keeping the slots
            void *np = nullptr;
            if (hipMalloc(&np, need + need / 8) != hipSuccess) return prgpu_oom("sw CIGAR spill", SB_CIG, need + need / 8);
            HIPCHK(hipMemcpyAsync(np, r.buf[SB_CIG], (size_t)r.cig_slots * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
            (void)hipFree(r.buf[SB_CIG]);
            prgpu_mem_note("sw", SB_CIG, (int64_t)(need + need / 8) - (int64_t)r.cap[SB_CIG]);
            r.buf[SB_CIG] = np;
            r.cap[SB_CIG] = need + need / 8;
            D.o_cig = (uint32_t *)np;
        }
        HIPCHK(hipMemsetAsync(D.work, 0, 4, s));
        e = sw_launch_overflow(D, O, grid_g, lds_glob, (void *)s);
        if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    }
    r.n_overflow = (int64_t)sp[0];
    HIPCHK(hipEventRecord(ctx_event(c, 0), s));
    return 0;
}

template <class T>
static int down(T *h, const SwResident &r, int id, size_t n, hipStream_t s) {
    if (h && n) HIPCHK(hipMemcpyAsync(h, r.buf[id], n * sizeof(T), hipMemcpyDeviceToHost, s));
    return 0;
}

// bwa mode: the per-task arrays gathered per reported alignment (SAM order) into SB_GDOWN
struct BwaRows {
    int32_t *qb, *qe, *rb, *re, *score, *truesc, *pos, *ncig, *status, *task;
    int64_t *cig_at;
    uint8_t *pass;
    int32_t *sr, *lr;   // the alignment's short read, long read and strand (its seed task's)
    uint8_t *strand;
};
static int bwa_gather(pr_ctx *c, SwResident &r, BwaRows &g) {
    hipStream_t s = ctx_stream(c);
    const int64_t n = r.n_aln;
    const size_t n1 = (size_t)n + 1;
    int rc;
    if ((rc = ensure(r, SB_GDOWN, n1 * (12 * 4 + 8 + 2) + 64))) return rc;
    char *b = (char *)r.buf[SB_GDOWN];
    int32_t **f[12] = {&g.qb, &g.qe, &g.rb, &g.re, &g.score, &g.truesc, &g.pos, &g.ncig, &g.status, &g.task, &g.sr, &g.lr};
    for (int k = 0; k < 12; ++k) *f[k] = (int32_t *)(b + (size_t)k * n1 * 4);
    g.cig_at = (int64_t *)(b + ((12 * n1 * 4 + 7) & ~(size_t)7));
    g.pass = (uint8_t *)(g.cig_at + n1);
    g.strand = g.pass + n1;
    SwGather G;
    std::memset(&G, 0, sizeof G);
    G.list = (const int32_t *)r.buf[SB_ALIST];
    G.n = n;
    G.t_sr = (const int32_t *)r.buf[SB_T_SR];
    G.t_lr = (const int32_t *)r.buf[SB_T_LR];
    G.status = (const int32_t *)r.buf[SB_STATUS];
    G.pos = (const int32_t *)r.buf[SB_POS];
    G.score = (const int32_t *)r.buf[SB_SCORE];
    G.ncig = (const int32_t *)r.buf[SB_NCIG];
    G.qb = (const int32_t *)r.buf[SB_QB];
    G.qe = (const int32_t *)r.buf[SB_QE];
    G.rb = (const int32_t *)r.buf[SB_RB];
    G.re = (const int32_t *)r.buf[SB_RE];
    G.truesc = (const int32_t *)r.buf[SB_TRUESC];
    G.pass = (const uint8_t *)r.buf[SB_PASS];
    G.cig_at = (const int64_t *)r.buf[SB_CIGAT];
    G.o_qb = g.qb; G.o_qe = g.qe; G.o_rb = g.rb; G.o_re = g.re; G.o_score = g.score; G.o_truesc = g.truesc;
    G.o_pos = g.pos; G.o_ncig = g.ncig; G.o_status = g.status; G.o_task = g.task; G.o_cig_at = g.cig_at;
    G.o_pass = g.pass;
    G.strand = (const uint8_t *)r.buf[SB_T_STRAND];
    G.o_sr = g.sr; G.o_lr = g.lr; G.o_strand = g.strand;
    const int e = sw_launch_gather(G, (void *)s);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    return 0;
}

static int bwa_download(pr_ctx *c, SwResident &r, pr_sw_out *o) {
    hipStream_t s = ctx_stream(c);
    BwaRows g;
    int rc;
    if ((rc = bwa_gather(c, r, g))) return rc;
    const size_t n = (size_t)r.n_aln;
    auto d32 = [&](int32_t *h, const int32_t *dv) -> int {
        if (h && n) HIPCHK(hipMemcpyAsync(h, dv, n * 4, hipMemcpyDeviceToHost, s));
        return 0;
    };
    if ((rc = d32(o->qb, g.qb)) || (rc = d32(o->qe, g.qe)) || (rc = d32(o->rb, g.rb)) || (rc = d32(o->re, g.re)) ||
        (rc = d32(o->score, g.score)) || (rc = d32(o->truesc, g.truesc)) || (rc = d32(o->pos, g.pos)) ||
        (rc = d32(o->ncigar, g.ncig)) || (rc = d32(o->status, g.status)) || (rc = d32(o->task, g.task)) ||
        (rc = d32(o->flag, (const int32_t *)r.buf[SB_AFLAG])))
        return rc;
    if (o->pass && n) HIPCHK(hipMemcpyAsync(o->pass, g.pass, n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!o->cigar_off && !o->cigar) return 0;
    std::vector<int32_t> nc(n + 1, 0), st(n + 1, 0);
    if (n) {
        HIPCHK(hipMemcpy(nc.data(), g.ncig, n * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(st.data(), g.status, n * 4, hipMemcpyDeviceToHost));
    }
    std::vector<int64_t> off(n + 1, 0);
    for (size_t t = 0; t < n; ++t) off[t + 1] = off[t] + (st[t] == 0 ? nc[t] : 0);
    if (o->cigar_off) std::memcpy(o->cigar_off, off.data(), (n + 1) * 8);
    if (!o->cigar) return 0;
    if (off[n] > o->cigar_cap) return pr_set_error(PR_ERR_CAPACITY, "pr_sw_out.cigar_cap below the CIGAR total");
    if (!off[n]) return 0;
    if ((rc = up(r, SB_CIGOFF, off.data(), n + 1, s)) || (rc = ensure(r, SB_CIGOUT, (size_t)off[n] * 4))) return rc;
    int e = sw_launch_cig_compact((const uint32_t *)r.buf[SB_CIG], g.cig_at, g.ncig, (const int64_t *)r.buf[SB_CIGOFF],
                                  (int64_t)n, (uint32_t *)r.buf[SB_CIGOUT], (void *)s);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    HIPCHK(hipMemcpyAsync(o->cigar, r.buf[SB_CIGOUT], (size_t)off[n] * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

extern "C" int pr_sw_download(pr_ctx *c, pr_sw_out *o) {
    if (!c || !o) return pr_set_error(PR_ERR_ARG, "null arg");
    SwResident &r = ctx_sw(c);
    HIPCHK(hipSetDevice(ctx_device(c)));
    hipStream_t s = ctx_stream(c);
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
    if (r.n_task) {
        float a = 0.f, b = 0.f;
        if (hipEventElapsedTime(&a, ctx_event(c, 2), ctx_event(c, 3)) == hipSuccess) r.ms_ext = a;
        if (hipEventElapsedTime(&b, ctx_event(c, 3), ctx_event(c, 0)) == hipSuccess) r.ms_glob = b;
        if (hipEventElapsedTime(&b, ctx_event(c, 6), ctx_event(c, 7)) == hipSuccess) r.ms_glob_ring = b;
    }
    HIPCHK(hipMemcpy(r.cells, r.buf[SB_CELLS], 24, hipMemcpyDeviceToHost));
    if (r.bwa) return bwa_download(c, r, o);
    const size_t n = (size_t)r.n_task;
    int rc;
    if ((rc = down(o->qb, r, SB_QB, n, s)) || (rc = down(o->qe, r, SB_QE, n, s)) ||
        (rc = down(o->rb, r, SB_RB, n, s)) || (rc = down(o->re, r, SB_RE, n, s)) ||
        (rc = down(o->score, r, SB_SCORE, n, s)) || (rc = down(o->truesc, r, SB_TRUESC, n, s)) ||
        (rc = down(o->pos, r, SB_POS, n, s)) || (rc = down(o->ncigar, r, SB_NCIG, n, s)) ||
        (rc = down(o->pass, r, SB_PASS, n, s)) || (rc = down(o->status, r, SB_STATUS, n, s)))
        return rc;
    HIPCHK(hipStreamSynchronize(s));
    if (!o->cigar_off && !o->cigar) return 0;
    // CIGARs: prefix of the op counts (status 0 tasks), then one compaction launch
    std::vector<int32_t> nc(n + 1, 0), st(n + 1, 0);
    if (n) {
        HIPCHK(hipMemcpy(nc.data(), r.buf[SB_NCIG], n * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(st.data(), r.buf[SB_STATUS], n * 4, hipMemcpyDeviceToHost));
    }
    std::vector<int64_t> off(n + 1, 0);
    for (size_t t = 0; t < n; ++t) off[t + 1] = off[t] + (st[t] == 0 ? nc[t] : 0);
    if (o->cigar_off) std::memcpy(o->cigar_off, off.data(), (n + 1) * 8);
    if (!o->cigar) return 0;
    if (off[n] > o->cigar_cap) return pr_set_error(PR_ERR_CAPACITY, "pr_sw_out.cigar_cap below the CIGAR total");
    if (!off[n]) return 0;
    if ((rc = up(r, SB_CIGOFF, off.data(), n + 1, s)) || (rc = ensure(r, SB_CIGOUT, (size_t)off[n] * 4))) return rc;
    int e = sw_launch_cig_compact((const uint32_t *)r.buf[SB_CIG], (const int64_t *)r.buf[SB_CIGAT],
                                  (const int32_t *)r.buf[SB_NCIG], (const int64_t *)r.buf[SB_CIGOFF], (int64_t)n,
                                  (uint32_t *)r.buf[SB_CIGOUT], (void *)s);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    HIPCHK(hipMemcpyAsync(o->cigar, r.buf[SB_CIGOUT], (size_t)off[n] * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

extern "C" int pr_sw_cigar_total(pr_ctx *c, int64_t *total, int64_t *n_overflow) {
    if (!c || !total) return pr_set_error(PR_ERR_ARG, "null arg");
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    HIPCHK(hipSetDevice(ctx_device(c)));
    HIPCHK(hipStreamSynchronize(ctx_stream(c)));
    const size_t n = (size_t)(r.bwa ? r.n_aln : r.n_task);
    std::vector<int32_t> nc(n + 1, 0), st(n + 1, 0);
    if (n && r.bwa) {
        BwaRows g;
        int rc = bwa_gather(c, r, g);
        if (rc) return rc;
        HIPCHK(hipStreamSynchronize(ctx_stream(c)));
        HIPCHK(hipMemcpy(nc.data(), g.ncig, n * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(st.data(), g.status, n * 4, hipMemcpyDeviceToHost));
    } else if (n) {
        HIPCHK(hipMemcpy(nc.data(), r.buf[SB_NCIG], n * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(st.data(), r.buf[SB_STATUS], n * 4, hipMemcpyDeviceToHost));
    }
    int64_t tot = 0;
    for (size_t t = 0; t < n; ++t) tot += st[t] == 0 ? nc[t] : 0;
    *total = tot;
    if (n_overflow) *n_overflow = r.n_overflow;
    return 0;
}

extern "C" int pr_sw_aln_count(pr_ctx *c, int64_t *n_aln) {
    if (!c || !n_aln) return pr_set_error(PR_ERR_ARG, "null arg");
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    HIPCHK(hipSetDevice(ctx_device(c)));
    HIPCHK(hipStreamSynchronize(ctx_stream(c)));
    *n_aln = r.bwa ? r.n_aln : r.n_task;
    return 0;
}

// pr_sw_binfilter's keep flags (computed per alignment in the long-read grouping of bwa_group,
// on the device) into SAM order: the grouping lists the alignments' tasks (SB_GLIST), SAM order
// lists them too (SB_ALIST), and a task reports at most one alignment
int sw_keep_to_sam(pr_ctx *c, const uint8_t *keep_grouped, uint8_t *keep_sam) {
    SwResident &r = ctx_sw(c);
    if (!r.loaded || !r.bwa) return pr_set_error(PR_ERR_ARG, "no resident bwa-mode SW batch");
    hipStream_t s = ctx_stream(c);
    const size_t n = (size_t)r.n_aln;
    std::vector<int32_t> gl(n + 1), al(n + 1);
    std::vector<uint8_t> kg(n + 1);
    if (n) {
        HIPCHK(hipMemcpyAsync(gl.data(), r.buf[SB_GLIST], n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(al.data(), r.buf[SB_ALIST], n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(kg.data(), keep_grouped, n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    std::vector<uint8_t> by_task((size_t)r.n_task + 1, 0);
    for (size_t j = 0; j < n; ++j) {
        if (gl[j] < 0 || gl[j] >= r.n_task) return pr_set_error(PR_ERR_ARG, "alignment grouping out of range");
        by_task[(size_t)gl[j]] = kg[j];
    }
    for (size_t i = 0; i < n; ++i) keep_sam[i] = by_task[(size_t)al[i]];
    return 0;
}

extern "C" int pr_sw_sam(pr_ctx *c, const pr_sam_in *in, char **text, int64_t *len, int64_t *n_records) {
    if (!c || !in || !text || !len || !in->sr_off || !in->sr_text || !in->sr_names || !in->sr_name_off ||
        !in->lr_names || !in->lr_name_off)
        return pr_set_error(PR_ERR_ARG, "null arg");
    *text = nullptr;
    *len = 0;
    SwResident &r = ctx_sw(c);
    if (!r.loaded || !r.bwa) return pr_set_error(PR_ERR_ARG, "no resident bwa-mode SW batch (pr_sw_launch first)");
    HIPCHK(hipSetDevice(ctx_device(c)));
    hipStream_t s = ctx_stream(c);
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
    const size_t n = (size_t)r.n_aln;
    BwaRows g;
    int rc;
    if ((rc = bwa_gather(c, r, g))) return rc;
    std::vector<int32_t> pos(n + 1), score(n + 1), ncig(n + 1), st(n + 1), sr(n + 1), lr(n + 1), flag(n + 1);
    std::vector<uint8_t> pass(n + 1), strand(n + 1);
    auto d32 = [&](std::vector<int32_t> &h, const void *dv) -> int {
        if (n) HIPCHK(hipMemcpyAsync(h.data(), dv, n * 4, hipMemcpyDeviceToHost, s));
        return 0;
    };
    if ((rc = d32(pos, g.pos)) || (rc = d32(score, g.score)) || (rc = d32(ncig, g.ncig)) || (rc = d32(st, g.status)) ||
        (rc = d32(sr, g.sr)) || (rc = d32(lr, g.lr)) || (rc = d32(flag, r.buf[SB_AFLAG])))
        return rc;
    if (n) {
        HIPCHK(hipMemcpyAsync(pass.data(), g.pass, n, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(strand.data(), g.strand, n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    // the printed alignments' CIGARs, compacted on the device
    std::vector<int64_t> off(n + 1, 0);
    for (size_t t = 0; t < n; ++t) {
        const bool pr = st[t] == 0 && pass[t] && (!in->keep || in->keep[t]);
        off[t + 1] = off[t] + (pr ? ncig[t] : 0);
        if (!pr) ncig[t] = -1;
    }
    std::vector<uint32_t> cig((size_t)off[n] + 1);
    if (off[n]) {
        std::vector<int32_t> nc_dev(n);
        for (size_t t = 0; t < n; ++t) nc_dev[t] = ncig[t] < 0 ? 0 : ncig[t];
        if ((rc = up(r, SB_CIGOFF, off.data(), n + 1, s)) || (rc = ensure(r, SB_CIGOUT, (size_t)off[n] * 4))) return rc;
        // the compaction reads its op counts from the device: the printed ones, 0 for the rest
        HIPCHK(hipMemcpyAsync(g.ncig, nc_dev.data(), n * 4, hipMemcpyHostToDevice, s));
        const int e = sw_launch_cig_compact((const uint32_t *)r.buf[SB_CIG], g.cig_at, g.ncig,
                                            (const int64_t *)r.buf[SB_CIGOFF], (int64_t)n, (uint32_t *)r.buf[SB_CIGOUT],
                                            (void *)s);
        if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
        HIPCHK(hipMemcpyAsync(cig.data(), r.buf[SB_CIGOUT], (size_t)off[n] * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    const int64_t n_sr = r.n_sr, n_lr = r.n_lr;
    for (size_t t = 0; t < n; ++t)
        if (ncig[t] >= 0 && (sr[t] < 0 || sr[t] >= n_sr || lr[t] < 0 || lr[t] >= n_lr))
            return pr_set_error(PR_ERR_ARG, "pr_sw_sam: an alignment names a read outside the batch");
    // the records, formatted in parallel over ranges of alignments (SAM order kept): each
    // record's exact length first, then every thread writes its range straight into the one
    // output buffer at its prefix-summed offset (no growing strings, no serial concatenation)
    int nt = in->n_threads > 0 ? in->n_threads : (int)std::thread::hardware_concurrency();
    nt = nt < 1 ? 1 : (nt > 64 ? 64 : nt);
    if ((size_t)nt > n / 1024 + 1) nt = (int)(n / 1024 + 1);
    static const char OPS[] = "MIDNSHP=X";
    static const char CMP[] = "TGCAN";   // reverse complement of nt4 codes A0 C1 G2 T3 N4
    auto ndig = [](int64_t v) -> int64_t {
        int64_t d = v < 0 ? 2 : 1;
        uint64_t u = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
        while (u >= 10) u /= 10, ++d;
        return d;
    };
    auto put = [](char *p, int64_t v) -> char * {
        if (v < 0) *p++ = '-', v = -v;
        char tmp[24];
        int k = 0;
        do tmp[k++] = (char)('0' + v % 10), v /= 10; while (v);
        while (k) *p++ = tmp[--k];
        return p;
    };
    std::vector<int64_t> rlen(n + 1, 0), part((size_t)nt + 1, 0), nrec((size_t)nt, 0);
    auto range = [&](int k, size_t &t0, size_t &t1) {
        t0 = n * (size_t)k / (size_t)nt;
        t1 = n * (size_t)(k + 1) / (size_t)nt;
    };
    auto measure = [&](int k) {
        size_t t0, t1;
        range(k, t0, t1);
        int64_t sum = 0, nr = 0;
        for (size_t t = t0; t < t1; ++t) {
            if (ncig[t] < 0) continue;
            const int64_t ql = in->sr_off[sr[t] + 1] - in->sr_off[sr[t]];
            int64_t L = (in->sr_name_off[sr[t] + 1] - in->sr_name_off[sr[t]]) + 1 + ndig(flag[t]) + 1 +
                        (in->lr_name_off[lr[t] + 1] - in->lr_name_off[lr[t]]) + 1 + ndig((int64_t)pos[t] + 1) + 1 +
                        ((flag[t] & 0x100) ? 1 : 2) + 1;
            for (int64_t x = off[t]; x < off[t + 1]; ++x) L += ndig(cig[(size_t)x] >> 4) + 1;
            L += 7 + ql + 1 + (in->sr_qual ? ql : 1) + 6 + ndig(score[t]) + 1;
            rlen[t] = L;
            sum += L;
            ++nr;
        }
        part[(size_t)k + 1] = sum;
        nrec[(size_t)k] = nr;
    };
    char *buf = nullptr;
    auto write = [&](int k) {
        size_t t0, t1;
        range(k, t0, t1);
        char *p = buf + part[(size_t)k];
        for (size_t t = t0; t < t1; ++t) {
            if (ncig[t] < 0) continue;
            char *const rec = p;
            const int64_t q0 = in->sr_off[sr[t]], q1 = in->sr_off[sr[t] + 1];
            const int64_t sn = in->sr_name_off[sr[t] + 1] - in->sr_name_off[sr[t]];
            std::memcpy(p, in->sr_names + in->sr_name_off[sr[t]], (size_t)sn);
            p += sn;
            *p++ = '\t';
            p = put(p, flag[t]);
            *p++ = '\t';
            const int64_t ln = in->lr_name_off[lr[t] + 1] - in->lr_name_off[lr[t]];
            std::memcpy(p, in->lr_names + in->lr_name_off[lr[t]], (size_t)ln);
            p += ln;
            *p++ = '\t';
            p = put(p, (int64_t)pos[t] + 1);
            *p++ = '\t';
            p = put(p, (flag[t] & 0x100) ? 0 : 60);
            *p++ = '\t';
            for (int64_t x = off[t]; x < off[t + 1]; ++x) {
                p = put(p, cig[(size_t)x] >> 4);
                *p++ = OPS[cig[(size_t)x] & 15u];
            }
            std::memcpy(p, "\t*\t0\t0\t", 7);
            p += 7;
            if (strand[t]) {
                for (int64_t x = q1 - 1; x >= q0; --x) {
                    const uint8_t b = in->sr_text[x] | 0x20;
                    *p++ = CMP[b == 'a' ? 0 : b == 'c' ? 1 : b == 'g' ? 2 : b == 't' ? 3 : 4];
                }
            } else {
                for (int64_t x = q0; x < q1; ++x) {
                    const uint8_t b = in->sr_text[x];
                    *p++ = (char)(b >= 'a' && b <= 'z' ? b - 32 : b);
                }
            }
            *p++ = '\t';
            if (!in->sr_qual) *p++ = '*';
            else if (strand[t])
                for (int64_t x = q1 - 1; x >= q0; --x) *p++ = (char)in->sr_qual[x];
            else {
                std::memcpy(p, in->sr_qual + q0, (size_t)(q1 - q0));
                p += q1 - q0;
            }
            std::memcpy(p, "\tAS:i:", 6);
            p += 6;
            p = put(p, score[t]);
            *p++ = '\n';
            if (p - rec != rlen[t]) std::abort();   // measure and write disagree: a bug here, never data
        }
    };
    auto run = [&](auto &&fn) {
        std::vector<std::thread> th;
        for (int k = 1; k < nt; ++k) th.emplace_back(fn, k);
        fn(0);
        for (auto &x : th) x.join();
    };
    run(measure);
    int64_t nr = 0;
    for (int k = 0; k < nt; ++k) part[(size_t)k + 1] += part[(size_t)k], nr += nrec[(size_t)k];
    const size_t tot = (size_t)part[(size_t)nt];
    buf = (char *)std::malloc(tot + 1);
    if (!buf) return pr_set_error(PR_ERR_ARG, "pr_sw_sam: out of host memory for the SAM text");
    run(write);
    buf[tot] = 0;
    *text = buf;
    *len = (int64_t)tot;
    if (n_records) *n_records = nr;
    return 0;
}

extern "C" int pr_sw_bwa_timing(pr_ctx *c, float *walk_ms, float *final_ms, float *early_final_ms) {
    if (!c) return pr_set_error(PR_ERR_ARG, "null ctx");
    SwResident &r = ctx_sw(c);
    if (walk_ms) *walk_ms = r.ms_walk;
    if (final_ms) *final_ms = r.ms_final;
    if (early_final_ms) *early_final_ms = r.ms_final_early;
    return 0;
}

extern "C" int pr_sw_bwa_stats(pr_ctx *c, int32_t *rounds, int64_t *n_extended, int64_t *n_patch) {
    if (!c) return pr_set_error(PR_ERR_ARG, "null ctx");
    SwResident &r = ctx_sw(c);
    if (rounds) *rounds = r.ext_rounds;
    if (n_extended) *n_extended = r.n_ext;
    if (n_patch) *n_patch = r.n_patch;
    return 0;
}

extern "C" int pr_sw_run(pr_ctx *c, const pr_sw_opts *o, const pr_sw_batch *b, pr_sw_out *out) {
    int rc = pr_sw_upload(c, b);
    if (rc) return rc;
    if ((rc = pr_sw_launch(c, o))) return rc;
    return pr_sw_download(c, out);
}

extern "C" int pr_sw_last_timing(pr_ctx *c, double *ms_extend, double *ms_global) {
    if (!c) return pr_set_error(PR_ERR_ARG, "null ctx");
    SwResident &r = ctx_sw(c);
    if (r.loaded && r.n_task) {   // from the launch's events (pipelines that never call pr_sw_download)
        HIPCHK(hipSetDevice(ctx_device(c)));
        HIPCHK(hipStreamSynchronize(ctx_stream(c)));
        float a = 0.f, b = 0.f;
        if (hipEventElapsedTime(&a, ctx_event(c, 2), ctx_event(c, 3)) == hipSuccess) r.ms_ext = a;
        if (hipEventElapsedTime(&b, ctx_event(c, 3), ctx_event(c, 0)) == hipSuccess) r.ms_glob = b;
        (void)hipGetLastError();
    }
    if (ms_extend) *ms_extend = r.ms_ext;
    if (ms_global) *ms_global = r.ms_glob;
    return 0;
}

extern "C" int pr_sw_last_cells(pr_ctx *c, int64_t *ce, int64_t *cg) {
    if (!c) return pr_set_error(PR_ERR_ARG, "null ctx");
    SwResident &r = ctx_sw(c);
    if (r.loaded && r.buf[SB_CELLS]) {
        HIPCHK(hipSetDevice(ctx_device(c)));
        HIPCHK(hipStreamSynchronize(ctx_stream(c)));
        HIPCHK(hipMemcpy(r.cells, r.buf[SB_CELLS], 24, hipMemcpyDeviceToHost));
    }
    if (ce) *ce = (int64_t)r.cells[0];
    if (cg) *cg = (int64_t)r.cells[1];
    return 0;
}

extern "C" int pr_sw_dominant_kernel(pr_ctx *c, double *ms, int64_t *cells) {
    // the CIGAR pass's register-ring launch (band <= 40): HIP events around that
    // launch alone on the SW stream, and the DP cells it computed
    if (!c) return pr_set_error(PR_ERR_ARG, "null ctx");
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    HIPCHK(hipSetDevice(ctx_device(c)));
    HIPCHK(hipStreamSynchronize(ctx_stream(c)));
    float b = 0.f;
    if (r.n_task && hipEventElapsedTime(&b, ctx_event(c, 6), ctx_event(c, 7)) == hipSuccess) r.ms_glob_ring = b;
    HIPCHK(hipMemcpy(r.cells, r.buf[SB_CELLS], 24, hipMemcpyDeviceToHost));
    if (ms) *ms = r.ms_glob_ring;
    if (cells) *cells = (int64_t)r.cells[2];
    return 0;
}

extern "C" int pr_sw_extension_kernels(pr_ctx *c, double *ms, int64_t *cells, int32_t *launches) {
    // every extension DP launch of the last pr_sw_launch (packed, ring, wide; all bwa-mode
    // rounds and both band tries): HIP events around each on the SW stream, summed, and the
    // DP cells they computed
    if (!c) return pr_set_error(PR_ERR_ARG, "null ctx");
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    HIPCHK(hipSetDevice(ctx_device(c)));
    HIPCHK(hipStreamSynchronize(ctx_stream(c)));
    double tot = 0.0;
    for (int i = 0; i + 1 < r.ext_ev.n; i += 2) {
        float a = 0.f;
        HIPCHK(hipEventElapsedTime(&a, (hipEvent_t)r.ext_ev.ev[i], (hipEvent_t)r.ext_ev.ev[i + 1]));
        tot += a;
    }
    HIPCHK(hipMemcpy(r.cells, r.buf[SB_CELLS], 24, hipMemcpyDeviceToHost));
    if (ms) *ms = tot;
    if (cells) *cells = (int64_t)r.cells[0];
    if (launches) *launches = r.ext_ev.n / 2;
    if (r.ext_ev.dropped) return pr_set_error(PR_ERR_CAPACITY, "more extension launches than timed events");
    return 0;
}

// for the SW -> consensus pipeline (prgpu_api.cpp)
// bwa mode: the reported alignments regrouped by long read (stable) and gathered into the
// per-task arrays the hand-off reads (SB_GPIPE), with task_off on the device
static int bwa_group(pr_ctx *c, SwResident &r, SwPtrs *p) {
    hipStream_t s = ctx_stream(c);
    const int64_t n = r.n_aln;
    const size_t n1 = (size_t)n + 1, l1 = (size_t)r.n_lr + 1;
    int rc;
    if ((rc = ensure(r, SB_GLIST, n1 * 4)) || (rc = ensure(r, SB_GKEY0, n1 * 4)) || (rc = ensure(r, SB_GKEY1, n1 * 4)) ||
        (rc = ensure(r, SB_GCNT, l1 * 4)) || (rc = ensure(r, SB_GLROFF, l1 * 8)) ||
        (rc = ensure(r, SB_GPIPE, n1 * (6 * 4 + 8 + 2) + 64)) || (rc = ensure(r, SB_SCANIN, (l1 + n1) * 8)))
        return rc;
    size_t tb = aln_group_temp_bytes(n, (int32_t)r.n_lr);
    if (tb > r.cap[SB_ATEMP] && (rc = ensure(r, SB_ATEMP, tb))) return rc;
    int e = aln_launch_group_lr((const int32_t *)r.buf[SB_ALIST], (const int32_t *)r.buf[SB_T_LR], n, (int32_t)r.n_lr,
                                (int32_t *)r.buf[SB_GKEY0], (int32_t *)r.buf[SB_GKEY1], (int32_t *)r.buf[SB_GLIST],
                                (int32_t *)r.buf[SB_GCNT], (int64_t *)r.buf[SB_GLROFF], (int64_t *)r.buf[SB_SCANIN],
                                r.buf[SB_ATEMP], r.cap[SB_ATEMP], (void *)s);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    char *b = (char *)r.buf[SB_GPIPE];
    int32_t *o32[6];
    for (int k = 0; k < 6; ++k) o32[k] = (int32_t *)(b + (size_t)k * n1 * 4);
    int64_t *cig_at = (int64_t *)(b + ((6 * n1 * 4 + 7) & ~(size_t)7));
    uint8_t *strand = (uint8_t *)(cig_at + n1), *pass = strand + n1;
    SwGather G;
    std::memset(&G, 0, sizeof G);
    G.list = (const int32_t *)r.buf[SB_GLIST];
    G.n = n;
    G.t_sr = (const int32_t *)r.buf[SB_T_SR];
    G.t_lr = (const int32_t *)r.buf[SB_T_LR];
    G.status = (const int32_t *)r.buf[SB_STATUS];
    G.pos = (const int32_t *)r.buf[SB_POS];
    G.score = (const int32_t *)r.buf[SB_SCORE];
    G.ncig = (const int32_t *)r.buf[SB_NCIG];
    G.strand = (const uint8_t *)r.buf[SB_T_STRAND];
    G.pass = (const uint8_t *)r.buf[SB_PASS];
    G.cig_at = (const int64_t *)r.buf[SB_CIGAT];
    G.o_sr = o32[0]; G.o_lr = o32[1]; G.o_status = o32[2]; G.o_pos = o32[3]; G.o_score = o32[4]; G.o_ncig = o32[5];
    G.o_cig_at = cig_at;
    G.o_strand = strand;
    G.o_pass = pass;
    if ((e = sw_launch_gather(G, (void *)s))) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    std::vector<int32_t> cnt(l1, 0);
    HIPCHK(hipMemcpyAsync(cnt.data(), r.buf[SB_GCNT], l1 * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int mx = 0;
    for (int64_t i = 0; i < r.n_lr; ++i) mx = cnt[(size_t)i] > mx ? cnt[(size_t)i] : mx;
    p->t_sr = o32[0];
    p->t_lr = o32[1];
    p->status = o32[2];
    p->pos = o32[3];
    p->score = o32[4];
    p->ncig = o32[5];
    p->cig_at = cig_at;
    p->strand = strand;
    p->pass = pass;
    p->n_task = n;
    p->task_off = (const int64_t *)r.buf[SB_GLROFF];
    p->max_per_lr = mx;
    return 0;
}

// the exchange's view of the last bwa-mode launch: the reported alignments (SAM order) and the
// per-task arrays they index (xchg_kernels.hip)
int sw_xchg_send(pr_ctx *c, XchgSend *X) {
    SwResident &r = ctx_sw(c);
    if (!r.loaded || !r.bwa) return pr_set_error(PR_ERR_ARG, "no resident bwa-mode SW launch (pr_sw_launch first)");
    X->n = r.n_aln;
    X->alist = (const int32_t *)r.buf[SB_ALIST];
    X->t_sr = (const int32_t *)r.buf[SB_T_SR];
    X->t_lr = (const int32_t *)r.buf[SB_T_LR];
    X->status = (const int32_t *)r.buf[SB_STATUS];
    X->pos = (const int32_t *)r.buf[SB_POS];
    X->score = (const int32_t *)r.buf[SB_SCORE];
    X->ncig = (const int32_t *)r.buf[SB_NCIG];
    X->strand = (const uint8_t *)r.buf[SB_T_STRAND];
    X->pass = (const uint8_t *)r.buf[SB_PASS];
    X->cig_at = (const int64_t *)r.buf[SB_CIGAT];
    X->cig = (const uint32_t *)r.buf[SB_CIG];
    return 0;
}

int sw_get_ptrs(pr_ctx *c, SwPtrs *p) {
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    p->task_off = nullptr;
    p->max_per_lr = 0;
    p->sr = (const uint8_t *)r.buf[SB_SR];
    p->lr = lr_pool(r);
    p->strand = (const uint8_t *)r.buf[SB_T_STRAND];
    p->pass = (const uint8_t *)r.buf[SB_PASS];
    p->sr_off = (const int64_t *)r.buf[SB_SR_OFF];
    p->lr_off = (const int64_t *)r.buf[SB_LR_OFF];
    p->t_sr = (const int32_t *)r.buf[SB_T_SR];
    p->t_lr = (const int32_t *)r.buf[SB_T_LR];
    p->status = (const int32_t *)r.buf[SB_STATUS];
    p->pos = (const int32_t *)r.buf[SB_POS];
    p->score = (const int32_t *)r.buf[SB_SCORE];
    p->ncig = (const int32_t *)r.buf[SB_NCIG];
    p->cig = (const uint32_t *)r.buf[SB_CIG];
    p->cig_at = (const int64_t *)r.buf[SB_CIGAT];
    p->n_task = r.n_task;
    p->n_sr = (int)r.n_sr;
    p->n_lr = (int)r.n_lr;
    return 0;
}

// the hand-off's view of the SW output: per task, or (bwa mode) the reported alignments grouped
// by long read (regrouped on the first call after a launch)
int sw_get_pipe_ptrs(pr_ctx *c, SwPtrs *p, bool regroup) {
    int rc = sw_get_ptrs(c, p);
    if (rc) return rc;
    SwResident &r = ctx_sw(c);
    if (!r.bwa) return 0;
    if (regroup) return bwa_group(c, r, p);
    const int64_t n = r.n_aln;
    const size_t n1 = (size_t)n + 1;
    char *b = (char *)r.buf[SB_GPIPE];
    p->t_sr = (const int32_t *)b;
    p->t_lr = (const int32_t *)(b + n1 * 4);
    p->status = (const int32_t *)(b + 2 * n1 * 4);
    p->pos = (const int32_t *)(b + 3 * n1 * 4);
    p->score = (const int32_t *)(b + 4 * n1 * 4);
    p->ncig = (const int32_t *)(b + 5 * n1 * 4);
    p->cig_at = (const int64_t *)(b + ((6 * n1 * 4 + 7) & ~(size_t)7));
    p->strand = (const uint8_t *)(p->cig_at + n1);
    p->pass = p->strand + n1;
    p->n_task = n;
    p->task_off = (const int64_t *)r.buf[SB_GLROFF];
    return 0;
}

extern "C" int pr_sw_phase_cycles(pr_ctx *c, int64_t *out4) {
    // wave-cycle totals of the packed CIGAR kernel's phases (masks, DP, backtrack, emit)
    if (!c || !out4) return pr_set_error(PR_ERR_ARG, "null arg");
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    HIPCHK(hipSetDevice(ctx_device(c)));
    HIPCHK(hipStreamSynchronize(ctx_stream(c)));
    unsigned long long v[10];
    HIPCHK(hipMemcpy(v, r.buf[SB_CELLS], sizeof v, hipMemcpyDeviceToHost));
    for (int q = 0; q < 4; ++q) out4[q] = (int64_t)v[3 + q];
    if (getenv("PRGPU_SW_DEBUG") && (atoi(getenv("PRGPU_SW_DEBUG")) & 4))   // backtrack walk statistics
        fprintf(stderr, "[sw] backtrack: %llu walk steps, %llu off-pair loads\n", v[9], v[7]);
    return 0;
}
