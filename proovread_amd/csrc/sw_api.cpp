// Host side of the SW stage C-ABI (include/prgpu.h pr_sw_*).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/prgpu.h"
#include "sw_dev.h"
#include "sw_pk.h"

using namespace prgpu;

// accessors defined in prgpu_api.cpp
SwResident &ctx_sw(pr_ctx *c);
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

namespace prgpu {
void sw_release(SwResident &r) {
    for (int i = 0; i < 40; ++i) {
        if (r.buf[i]) (void)hipFree(r.buf[i]);
        r.buf[i] = nullptr;
        r.cap[i] = 0;
    }
    r.loaded = false;
}
}  // namespace prgpu

static int ensure(SwResident &r, int id, size_t bytes) {
    if (r.buf[id] && r.cap[id] >= bytes) return 0;
    if (r.buf[id]) (void)hipFree(r.buf[id]);
    r.buf[id] = nullptr;
    r.cap[id] = 0;
    const size_t want = bytes + 64;   // slack: kernels read whole dwords at the end of byte pools
    if (hipMalloc(&r.buf[id], want) != hipSuccess) return pr_set_error(PR_ERR_HIP, "hipMalloc failed (SW)");
    r.cap[id] = want;
    return 0;
}
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

extern "C" int pr_sw_upload(pr_ctx *c, const pr_sw_batch *b) {
    if (!c || !b) return pr_set_error(PR_ERR_ARG, "null arg");
    if (b->n_sr < 0 || b->n_lr < 0 || b->n_task < 0) return pr_set_error(PR_ERR_ARG, "negative sizes");
    HIPCHK(hipSetDevice(ctx_device(c)));
    SwResident &r = ctx_sw(c);
    hipStream_t s = ctx_stream(c);
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
    for (int64_t t = 0; t < b->n_task; ++t) {
        const int sr = b->t_sr[t], lr = b->t_lr[t];
        if (sr < 0 || sr >= b->n_sr || lr < 0 || lr >= b->n_lr)
            return pr_set_error(PR_ERR_ARG, "task references a missing read");
        const int64_t lq = b->sr_off[sr + 1] - b->sr_off[sr], L = b->lr_off[lr + 1] - b->lr_off[lr];
        if (b->t_slen[t] <= 0 || b->t_qbeg[t] < 0 || b->t_qbeg[t] + b->t_slen[t] > lq || b->t_rbeg[t] < 0 ||
            b->t_rbeg[t] + b->t_slen[t] > L)
            return pr_set_error(PR_ERR_ARG, "seed outside its reads");
    }
    const int64_t nt = b->n_task;
    int rc;
    if ((rc = up(r, SB_SR, b->sr_seq, (size_t)b->sr_off[b->n_sr], s)) ||
        (rc = up(r, SB_SR_OFF, b->sr_off, (size_t)b->n_sr + 1, s)) ||
        (rc = up(r, SB_LR, b->lr_seq, (size_t)b->lr_off[b->n_lr], s)) ||
        (rc = up(r, SB_LR_OFF, b->lr_off, (size_t)b->n_lr + 1, s)) || (rc = up(r, SB_T_SR, b->t_sr, nt, s)) ||
        (rc = up(r, SB_T_LR, b->t_lr, nt, s)) || (rc = up(r, SB_T_STRAND, b->t_strand, nt, s)) ||
        (rc = up(r, SB_T_QBEG, b->t_qbeg, nt, s)) || (rc = up(r, SB_T_RBEG, b->t_rbeg, nt, s)) ||
        (rc = up(r, SB_T_SLEN, b->t_slen, nt, s)))
        return rc;
    const size_t n4 = (size_t)(nt + 1) * 4;
    for (int id : {SB_QB, SB_QE, SB_RB, SB_RE, SB_SCORE, SB_TRUESC, SB_W, SB_GSCORE, SB_POS, SB_NCIG, SB_STATUS})
        if ((rc = ensure(r, id, n4))) return rc;
    if ((rc = ensure(r, SB_PERM, (size_t)(nt + 1) * 4)) || (rc = ensure(r, SB_BUCKET, (SW_NBUCKET + 16 + PK_SCAN + 1) * 4)) ||
        (rc = ensure(r, SB_X, (size_t)(nt + 1) * 4 * 12)) || (rc = ensure(r, SB_XTRY, (size_t)nt + 1)) ||
        (rc = ensure(r, SB_LIST, (size_t)(nt + 1 + (int64_t)PK_NB * PK_SEG) * 4)))
        return rc;
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
    D.tmax = r.qmax + 4 * o->w + 4;
    D.sr = (const uint8_t *)r.buf[SB_SR];
    D.sr_off = (const int64_t *)r.buf[SB_SR_OFF];
    D.lr = (const uint8_t *)r.buf[SB_LR];
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
    int rc;
    if ((rc = ensure(r, SB_Z, zb))) return rc;
    D.z = (uint8_t *)r.buf[SB_Z];
    HIPCHK(hipMemsetAsync(r.buf[SB_CELLS], 0, CELLS_BYTES, s));
    if (r.n_task == 0) return 0;
    HIPCHK(hipMemcpyAsync(r.buf[SB_CIGAT], r.buf[SB_CIGSLOT], (size_t)r.n_task * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipEventRecord(ctx_event(c, 2), s));
    int e = sw_launch_extend(D, O, ctx_ncu(c) * 16, grid_pk, (void *)s);
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));

    HIPCHK(hipEventRecord(ctx_event(c, 3), s));
    e = sw_launch_global(D, O, grid_w, grid_pk, grid_g, lds_glob, (void *)s, (void *)ctx_event(c, 6), (void *)ctx_event(c, 7));
    if (e) return pr_set_error(PR_ERR_HIP, hipGetErrorString((hipError_t)e));
    // CIGARs longer than their slots: recompute those tasks into the spill area
    unsigned long long sp[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(sp, D.spill, sizeof sp, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (sp[0]) {
        const size_t need = (size_t)(r.cig_slots + (int64_t)sp[1]) * 4;
        if (need > r.cap[SB_CIG]) {   // grow the pool, keeping the slots
            void *np = nullptr;
            if (hipMalloc(&np, need + need / 8) != hipSuccess) return pr_set_error(PR_ERR_HIP, "hipMalloc failed (CIGAR spill)");
            HIPCHK(hipMemcpyAsync(np, r.buf[SB_CIG], (size_t)r.cig_slots * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
            (void)hipFree(r.buf[SB_CIG]);
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
    const size_t n = (size_t)r.n_task;
    std::vector<int32_t> nc(n + 1, 0), st(n + 1, 0);
    if (n) {
        HIPCHK(hipMemcpy(nc.data(), r.buf[SB_NCIG], n * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(st.data(), r.buf[SB_STATUS], n * 4, hipMemcpyDeviceToHost));
    }
    int64_t tot = 0;
    for (size_t t = 0; t < n; ++t) tot += st[t] == 0 ? nc[t] : 0;
    *total = tot;
    if (n_overflow) *n_overflow = r.n_overflow;
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

// for the SW -> consensus pipeline (prgpu_api.cpp)
int sw_get_ptrs(pr_ctx *c, SwPtrs *p) {
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    p->sr = (const uint8_t *)r.buf[SB_SR];
    p->lr = (const uint8_t *)r.buf[SB_LR];
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

extern "C" int pr_sw_phase_cycles(pr_ctx *c, int64_t *out4) {
    // wave-cycle totals of the packed CIGAR kernel's phases (masks, DP, backtrack, emit)
    if (!c || !out4) return pr_set_error(PR_ERR_ARG, "null arg");
    SwResident &r = ctx_sw(c);
    if (!r.loaded) return pr_set_error(PR_ERR_ARG, "no resident SW batch");
    HIPCHK(hipSetDevice(ctx_device(c)));
    HIPCHK(hipStreamSynchronize(ctx_stream(c)));
    unsigned long long v[7];
    HIPCHK(hipMemcpy(v, r.buf[SB_CELLS], sizeof v, hipMemcpyDeviceToHost));
    for (int q = 0; q < 4; ++q) out4[q] = (int64_t)v[3 + q];
    return 0;
}
