// Host side of libprgpu.so: the C-ABI declared in include/prgpu.h.
// Device memory, one HIP stream per context, HIP events for kernel timing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/prgpu.h"
#include "cns_dev.h"
#include "sw_dev.h"
#include "pipe_dev.h"
#include "mask_dev.h"
#include "seed_dev.h"
#include "seed_index_dev.h"
#include "xchg_dev.h"

using namespace prgpu;
int sw_get_ptrs(pr_ctx *c, SwPtrs *p);
int sw_xchg_send(pr_ctx *c, XchgSend *X);
pr_ctx *comm_ctx(pr_comm *c);
int sw_get_pipe_ptrs(pr_ctx *c, SwPtrs *p, bool regroup);
int sw_upload_device_seeds(pr_ctx *c, const pr_sw_batch *b, const pr_seed_task *dev_tasks, const int64_t *seed_off_h,
                           const uint8_t *dev_sr = nullptr, const uint8_t *dev_lr = nullptr);

static thread_local std::string g_err;
static int set_error(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(x)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess)                                                            \
            return set_error(PR_ERR_HIP, "%s failed: %s", #x, hipGetErrorString(e_));    \
    } while (0)

extern "C" const char *pr_last_error(void) { return g_err.c_str(); }
extern "C" const char *pr_version(void) { return "prgpu 0.1.0 (gfx950)"; }

// ---------------------------------------------------------------------------
// device memory of the library's buffers (all contexts of the process), and PRGPU_MEM_TRACE=1:
// every growth to stderr with the buffer's group and index (sizing at scale)
std::atomic<int64_t> g_dev_bytes{0};
static bool mem_trace() {
    static const bool on = [] { const char *e = std::getenv("PRGPU_MEM_TRACE"); return e && *e && *e != '0'; }();
    return on;
}
// per-group accounting behind pr_mem_stats (groups are the DevBuf tags and "sw")
namespace {
struct MemGroup {
    char name[16];
    int64_t cur, peak, at_peak;
};
std::mutex g_mem_mu;
MemGroup g_mem[16];
int g_mem_n = 0;
int64_t g_mem_peak = 0;
}   // namespace
void prgpu_mem_note(const char *grp, int id, int64_t delta) {
    const int64_t tot = g_dev_bytes.fetch_add(delta) + delta;
    {
        std::lock_guard<std::mutex> lk(g_mem_mu);
        // "sw CIGAR spill" and the like count under their group's first word
        char key[16] = {};
        for (int i = 0; i < 15 && grp[i] && grp[i] != ' '; ++i) key[i] = grp[i];
        int k = 0;
        while (k < g_mem_n && std::strcmp(g_mem[k].name, key) != 0) ++k;
        if (k == g_mem_n && g_mem_n < 16) {
            std::memcpy(g_mem[k].name, key, 16);
            g_mem[k].cur = g_mem[k].peak = g_mem[k].at_peak = 0;
            ++g_mem_n;
        }
        if (k < g_mem_n) {
            g_mem[k].cur += delta;
            g_mem[k].peak = std::max(g_mem[k].peak, g_mem[k].cur);
        }
        if (tot > g_mem_peak) {
            g_mem_peak = tot;
            for (int j = 0; j < g_mem_n; ++j) g_mem[j].at_peak = g_mem[j].cur;
        }
    }
    if (mem_trace() && delta > 0)
        std::fprintf(stderr, "[prgpu mem] %s[%d] +%.1f MB -> %.2f GB\n", grp, id, delta / 1e6, tot / 1e9);
}

extern "C" int pr_mem_stats(int64_t *cur, int64_t *peak, pr_mem_group *groups, int cap, int *n_groups) {
    std::lock_guard<std::mutex> lk(g_mem_mu);
    if (cur) *cur = g_dev_bytes.load();
    if (peak) *peak = g_mem_peak;
    const int n = std::min(g_mem_n, std::max(cap, 0));
    for (int k = 0; groups && k < n; ++k) {
        std::memcpy(groups[k].name, g_mem[k].name, 16);
        groups[k].cur = g_mem[k].cur;
        groups[k].peak = g_mem[k].peak;
        groups[k].at_total_peak = g_mem[k].at_peak;
    }
    if (n_groups) *n_groups = g_mem_n;
    return 0;
}

extern "C" void pr_mem_reset_peak(void) {
    std::lock_guard<std::mutex> lk(g_mem_mu);
    g_mem_peak = g_dev_bytes.load();
    for (int k = 0; k < g_mem_n; ++k) g_mem[k].peak = g_mem[k].at_peak = g_mem[k].cur;
}
int prgpu_oom(const char *grp, int id, size_t want) {
    size_t fr = 0, total = 0;
    (void)hipMemGetInfo(&fr, &total);
    (void)hipGetLastError();
    return set_error(PR_ERR_HIP, "hipMalloc(%zu) failed (%s[%d]; the library holds %.2f GB, device free %.2f of %.2f GB)",
                     want, grp, id, g_dev_bytes.load() / 1e9, fr / 1e9, total / 1e9);
}

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    const char *grp = "buf";
    int id = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return 0;
        release();
        size_t want = bytes + 64;   // slack: kernels read whole dwords at the end of byte pools
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            return prgpu_oom(grp, id, want);
        }
        cap = want;
        prgpu_mem_note(grp, id, (int64_t)want);
        return 0;
    }
    void release() {
        if (p) {
            (void)hipFree(p);
            prgpu_mem_note(grp, id, -(int64_t)cap);
        }
        p = nullptr;
        cap = 0;
    }
    // grow to `bytes` keeping the first `used` bytes (stream-ordered copy, then synchronised)
    int grow_keep(size_t bytes, size_t used, hipStream_t s) {
        if (bytes <= cap && p) return 0;
        void *np = nullptr;
        const size_t want = bytes + bytes / 4 + 64;
        if (hipMalloc(&np, want) != hipSuccess) return prgpu_oom(grp, id, want);
        if (p && used) {
            if (hipMemcpyAsync(np, p, used, hipMemcpyDeviceToDevice, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
                (void)hipFree(np);
                return set_error(PR_ERR_HIP, "device copy failed (%s[%d] growth)", grp, id);
            }
        }
        release();
        p = np;
        cap = want;
        prgpu_mem_note(grp, id, (int64_t)want);
        return 0;
    }
    template <class T>
    T *as() const { return reinterpret_cast<T *>(p); }
};

enum CnsBufId {
    CB_LR_OFF, CB_REF_SEQ, CB_REF_QUAL, CB_IGN_OFF, CB_IGN, CB_ALN_OFF, CB_POS, CB_SCORE, CB_AFLAGS,
    CB_SEQ_OFF, CB_LSEQ, CB_CIG_OFF, CB_NCIG, CB_SEQ, CB_CIG,
    CB_A_ST, CB_A_LEN, CB_A_NC, CB_A_BIN, CB_A_CB, CB_A_CE, CB_A_SB, CB_A_RPOS, CB_A_END,
    CB_SORTED, CB_LST_SCORE, CB_LST_ALN, CB_KEPT, CB_BIN_OFF, CB_BIN_BASES, CB_WORK,
    CB_OUT_OFF, CB_CHIM_OFF, CB_STATUS, CB_SEQ_LEN, CB_TRACE_LEN, CB_NCIGAR, CB_NCHIM,
    CB_O_SEQ, CB_O_QUAL, CB_O_TRACE, CB_O_CIG, CB_O_CHIM, CB_PROF, CB_RETRY, CB_K,
    CB_GSZS, CB_GSZC, CB_GSO, CB_GCO, CB_GTMP,
    CB_COUNT
};

// masking buffers (pr_mask_run inputs / outputs, pr_iter_mask output and run lists)
enum MaskBufId { MB_OFF, MB_SEQ, MB_QUAL, MB_OUT, MB_RUN_OFF, MB_RUNS, MB_TMP, MB_NRUNS, MB_ERR, MB_STATS, MB_COUNT };
// device seeding: the index copy (SI_*) and per-call buffers (SB_*)
enum SeedBufId {
    SI_TEXT, SI_CSTART, SI_CBLK, SI_LROFF, SI_KOFF, SI_KPOS, SI_KEXT, SI_CNT0,
    SB_SEQ = SI_CNT0 + 11, SB_OFF, SB_SCRATCH, SB_OUT, SB_NOUT, SB_STATUS, SB_NEXT, SB_PRE, SB_DENSE,
    SX_LRSEQ, SX_KEY0, SX_KEY1, SX_VAL0, SX_KC, SX_CNTPTR, SX_TEMP, SI_KSPLIT, SX_VAL1, SX_KCC, SX_KOFFC, SX_KCUR,
    SB_DP, SI_TEXT4, SB_ORDER, SI_BLKFR, SD_COUNT
};
// the exact-parity layout's exchange (pr_aln_exchange, owned batches): bounds, sort keys and
// indices, counts, op prefix, send / receive records and CIGAR ops, grouped hand-off inputs,
// the task's short reads
// the resident long-read set: pools, the dense offsets of a commit, the commit's staging pools
// (LS_RSEQ / LS_RQUAL: pr_lrset_snapshot's raw reads; LS_SRSAMP: pr_srset_sample's task sample)
enum LrSetBufId {
    LS_SEQ, LS_QUAL, LS_MAP, LS_OFF, LS_TSEQ, LS_TQUAL, LS_TMAP, LS_SRSEQ, LS_GSEQ, LS_GQUAL, LS_GMAP, LS_RSEQ, LS_RQUAL,
    LS_SRSAMP, LS_COUNT
};
enum XchgBufId {
    XB_BOUNDS, XB_KEY0, XB_KEY1, XB_IDX0, XB_IDX1, XB_CNT, XB_OPIN, XB_OPAT, XB_SREC, XB_SCIG, XB_TEMP,
    XB_RREC, XB_RCIG, XB_RCIGAT, XB_GCNT, XB_GCNT64, XB_TASKOFF, XB_ERR, XB_GSR, XB_GSTATUS, XB_GPOS, XB_GSCORE,
    XB_GNCIG, XB_GCIGAT, XB_GSTRAND, XB_GPASS, XB_SR, XB_SROFF, XB_COUNT
};

struct pr_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    hipEvent_t ev[11] = {};   // 0-7: SW, consensus, pipeline; 8-10: seeding
    // consensus resident batch
    DevBuf cb[CB_COUNT];
    bool cns_loaded = false;
    int32_t n_lr = 0;
    int64_t n_aln = 0, total_cols = 0, n_bins = 0, seq_cap = 0, chim_cap = 0;
    int64_t seed_pass2 = 0;   // reads of the last pr_seed_gpu_map that needed the large slices
    int64_t seed_pass3 = 0;   // ... and the grown slices of the later passes (counted per pass)
    std::vector<int64_t> seed_pre;   // per-read prefix of the last pr_seed_gpu_map's seeds (SB_DENSE)
    int64_t alg_bytes = 0;
    int64_t k_need = 0;   // per-read bound of kept alignments (K pool slices)
    bool has_ref = false, has_qual = false, has_ign = false;
    std::vector<int64_t> out_off, chim_off, bin_off, lr_off_host;
    float last_ms = 0.f;
    // SW -> consensus pipeline (pr_iter_*)
    bool pipe = false;
    bool pipe_ref_ascii = false;   // pr_iter_batch.ref_seq given: consensus reference in CB_REF_SEQ
    int pipe_sort_cap = 0;
    DevBuf pb[12];          // task_off, cnt, err, then the -b/-l filter: keep, sorted, bin, nc, len, lists
    float ms_pipe = 0.f, ms_cns = 0.f;
    // SW resident batch
    SwResident sw;
    // masking
    DevBuf mb[MB_COUNT];
    // seeding
    DevBuf sd[SD_COUNT];
    bool seed_loaded = false;
    seedc::IndexView seed_view{};
    float ms_seed = 0.f, ms_seed_pass2 = 0.f;
    float ms_index = 0.f;
    int64_t seed_n_text = 0, seed_n_hits = 0;
    int64_t seed_sr_bases = -1;   // bases of the short reads of the last pr_seed_gpu_map (SB_SEQ)
    bool iter_masked = false;
    bool cns_launched = false;   // a consensus launch filled the CB_O_* outputs
    bool cns_gathered = false;   // the hand-off's SEQ / CIGAR offsets point into CB_SEQ / CB_CIG
    // exact-parity layout: received alignments (pr_aln_exchange) and an owned batch
    DevBuf xb[XB_COUNT];
    bool x_ready = false;        // XB_RREC / XB_RCIG hold the last exchange's records
    bool x_pass = false;         // world 1: the exchange is the identity, the owned launch reads the SW output
    int64_t x_nrecv = 0, x_nrcig = 0;
    std::vector<int64_t> x_from;  // records of the last exchange by source rank
    // the resident long-read set (pr_lrset_*): reads, qualities, mapping reference (masked reads)
    DevBuf ls[LS_COUNT];
    std::vector<int64_t> ls_off;
    int32_t ls_n = -1;
    bool ls_map_is_reads = true;
    std::vector<int64_t> ss_off;   // the resident short reads (pr_srset_load): offsets on the host
    std::vector<int64_t> ss_samp_off;   // pr_srset_sample's task sample (LS_SRSAMP), empty: none
    std::vector<int64_t> ls_raw_off;    // pr_lrset_snapshot's offsets, empty: none
    bool seed_sr_staged = false;   // SB_SEQ already holds the reads of the next pr_seed_gpu_map
    bool own = false;            // the resident iteration batch is an owned batch (pr_iter_upload_owned)
    bool own_ref_nt4 = false;    // its consensus reference is the SW long-read pool's slice (nt4)
    bool own_sr_resident = false;   // its short reads are the resident ones (LS_SRSEQ)
    int32_t own_lr0 = 0;
};

extern "C" int pr_device_count(int *n) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return 0;
}

extern "C" int pr_ctx_create(int device, pr_ctx **out) {
    if (!out) return set_error(PR_ERR_ARG, "null out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return set_error(PR_ERR_HIP, "no HIP device visible (libprgpu needs an MI355X)");
    if (device < 0) HIPCHK(hipGetDevice(&device));
    if (device >= n) return set_error(PR_ERR_ARG, "device %d >= count %d", device, n);
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(PR_ERR_HIP, "device %d is %s, libprgpu is built for gfx950", device, prop.gcnArchName);
    pr_ctx *c = new pr_ctx();
    c->device = device;
    auto tag = [](DevBuf *b, int n, const char *g) {
        for (int i = 0; i < n; ++i) b[i].grp = g, b[i].id = i;
    };
    tag(c->cb, CB_COUNT, "cns");
    tag(c->pb, 12, "pipe");
    tag(c->mb, MB_COUNT, "mask");
    tag(c->sd, SD_COUNT, "seed");
    tag(c->xb, XB_COUNT, "xchg");
    tag(c->ls, LS_COUNT, "lrset");
    c->n_cu = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_error(PR_ERR_HIP, "hipStreamCreate failed");
    }
    for (auto &e : c->ev) (void)hipEventCreate(&e);
    *out = c;
    return 0;
}

extern "C" void pr_ctx_destroy(pr_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (auto &b : c->cb) b.release();
    for (auto &b : c->pb) b.release();
    for (auto &b : c->mb) b.release();
    for (auto &b : c->sd) b.release();
    for (auto &b : c->xb) b.release();
    for (auto &b : c->ls) b.release();
    sw_release(c->sw);
    for (auto &e : c->ev) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// ---------------------------------------------------------------------------
// consensus
extern "C" void pr_cns_params_default(pr_cns_params *p) {
    p->max_coverage = 50.0;  // Seq.pm:116 default; proovread passes --coverage
    p->bin_size = 20.0;
    p->trim = 1;
    p->indel_taboo_length = 7;
    p->indel_taboo = 0.1;
    p->min_aln_length = 50;
    p->max_ins_length = 0;
    p->fallback_phred = 1;
    p->phred_offset = 33;
    p->ref_phred_offset = 33;
    p->use_ref_qual = 1;
    p->qual_weighted = 0;
    p->detect_chimera = 0;
    p->invert_scores = 0;
}

static int validate_batch(const pr_cns_batch *b) {
    if (!b || b->n_lr < 0) return set_error(PR_ERR_ARG, "null batch");
    if (b->n_lr == 0) return 0;
    if (!b->lr_off || !b->aln_off) return set_error(PR_ERR_ARG, "lr_off/aln_off required");
    if (b->lr_off[0] != 0 || b->aln_off[0] != 0) return set_error(PR_ERR_ARG, "offsets must start at 0");
    for (int i = 0; i < b->n_lr; ++i) {
        if (b->lr_off[i + 1] < b->lr_off[i] || b->aln_off[i + 1] < b->aln_off[i])
            return set_error(PR_ERR_ARG, "offsets not monotone at %d", i);
        if (b->ign_off && b->ign_off[i + 1] < b->ign_off[i]) return set_error(PR_ERR_ARG, "ign_off not monotone");
    }
    const int64_t na = b->aln_off[b->n_lr];
    if (na && (!b->aln_pos || !b->aln_score || !b->aln_flags || !b->aln_seq_off || !b->aln_lseq ||
               !b->aln_cig_off || !b->aln_ncig || !b->cig_pool))
        return set_error(PR_ERR_ARG, "alignment arrays required");
    for (int64_t a = 0; a < na; ++a) {
        if (b->aln_cig_off[a] < 0 || b->aln_ncig[a] < 0 || b->aln_cig_off[a] + b->aln_ncig[a] > b->cig_pool_len)
            return set_error(PR_ERR_ARG, "cigar out of pool at alignment %lld", (long long)a);
        if (!(b->aln_flags[a] & PR_ALN_NO_SEQ) &&
            (b->aln_seq_off[a] < 0 || b->aln_lseq[a] < 0 || b->aln_seq_off[a] + b->aln_lseq[a] > b->seq_pool_len))
            return set_error(PR_ERR_ARG, "seq out of pool at alignment %lld", (long long)a);
    }
    return 0;
}

// Output capacities per long read (shared by pr_cns_bounds_of and the upload):
// consensus bytes <= L + inserted bases of all its alignments (+1); chimera
// records <= bins/2 + 2 (bins at the smallest bin size bam2cns uses, 20).
static void cns_caps(const pr_cns_batch *b, std::vector<int64_t> &out_off, std::vector<int64_t> &chim_off,
                     int64_t *in_bytes, int64_t *k_need = nullptr) {
    const int n = b->n_lr;
    out_off.assign(n + 1, 0);
    chim_off.assign(n + 1, 0);
    int64_t ib = 0, kmax = 0;
    for (int i = 0; i < n; ++i) {
        const int64_t L = b->lr_off[i + 1] - b->lr_off[i];
        int64_t ins = 0;
        for (int64_t a = b->aln_off[i]; a < b->aln_off[i + 1]; ++a) {
            ib += (b->aln_flags[a] & PR_ALN_NO_SEQ ? 0 : b->aln_lseq[a]) + 4 * (int64_t)b->aln_ncig[a] + 16;
            for (int k = 0; k < b->aln_ncig[a]; ++k) {
                const uint32_t cc = b->cig_pool[b->aln_cig_off[a] + k];
                if ((cc & 15u) == 1u) ins += cc >> 4;
            }
        }
        if (b->aln_off[i + 1] - b->aln_off[i] > kmax) kmax = b->aln_off[i + 1] - b->aln_off[i];
        const int64_t nb = (int64_t)((double)L / 20.0) + 1;
        out_off[i + 1] = out_off[i] + L + ins + 1;
        chim_off[i + 1] = chim_off[i] + nb / 2 + 2;
    }
    if (in_bytes) *in_bytes = ib;
    if (k_need) *k_need = kmax;
}

extern "C" int pr_cns_bounds_of(const pr_cns_batch *b, pr_cns_bounds *out) {
    int rc = validate_batch(b);
    if (rc) return rc;
    std::vector<int64_t> oo, co;
    cns_caps(b, oo, co, nullptr);
    out->seq_cap = oo.back();
    out->chim_cap = co.back();
    return 0;
}

template <class T>
static int upload(DevBuf &d, const T *h, size_t n, hipStream_t s) {
    int rc = d.ensure(n * sizeof(T));
    if (rc) return rc;
    if (n && h) HIPCHK(hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s));
    return 0;
}

extern "C" int pr_cns_upload(pr_ctx *c, const pr_cns_batch *b) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    int rc = validate_batch(b);
    if (rc) return rc;
    c->cns_launched = false;
    c->iter_masked = false;
    c->own = false;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const int n = b->n_lr;
    const int64_t na = n ? b->aln_off[n] : 0;
    const int64_t tl = n ? b->lr_off[n] : 0;
    c->n_lr = n;
    c->n_aln = na;
    c->total_cols = tl;
    c->pipe = false;
    c->lr_off_host.assign(b->lr_off, b->lr_off + n + 1);
    c->has_ref = b->ref_seq != nullptr;
    c->has_qual = b->ref_qual != nullptr;
    c->has_ign = b->ign_off != nullptr;
    int64_t in_bytes = 0;
    cns_caps(b, c->out_off, c->chim_off, &in_bytes, &c->k_need);
    c->seq_cap = c->out_off[n];
    c->chim_cap = c->chim_off[n];
    // SURVEY.md §8d pileup byte model: alignments in + ref seq/qual in + consensus out + state counts
    c->alg_bytes = in_bytes + tl * 2 + tl * 2 + tl * 6 * 4 * 2;

    DevBuf *B = c->cb;
    if ((rc = upload(B[CB_LR_OFF], b->lr_off, n + 1, s))) return rc;
    if ((rc = upload(B[CB_REF_SEQ], b->ref_seq, b->ref_seq ? tl : 0, s))) return rc;
    if ((rc = upload(B[CB_REF_QUAL], b->ref_qual, b->ref_qual ? tl : 0, s))) return rc;
    if (b->ign_off) {
        if ((rc = upload(B[CB_IGN_OFF], b->ign_off, n + 1, s))) return rc;
        if ((rc = upload(B[CB_IGN], b->ign, 2 * b->ign_off[n], s))) return rc;
    }
    if ((rc = upload(B[CB_ALN_OFF], b->aln_off, n + 1, s))) return rc;
    if ((rc = upload(B[CB_POS], b->aln_pos, na, s))) return rc;
    if ((rc = upload(B[CB_SCORE], b->aln_score, na, s))) return rc;
    if ((rc = upload(B[CB_AFLAGS], b->aln_flags, na, s))) return rc;
    if ((rc = upload(B[CB_SEQ_OFF], b->aln_seq_off, na, s))) return rc;
    if ((rc = upload(B[CB_LSEQ], b->aln_lseq, na, s))) return rc;
    if ((rc = upload(B[CB_CIG_OFF], b->aln_cig_off, na, s))) return rc;
    if ((rc = upload(B[CB_NCIG], b->aln_ncig, na, s))) return rc;
    if ((rc = upload(B[CB_SEQ], b->seq_pool, b->seq_pool_len, s))) return rc;
    if ((rc = upload(B[CB_CIG], b->cig_pool, b->cig_pool_len, s))) return rc;
    // per-alignment scratch
    const size_t na1 = (size_t)na + 1;
    if ((rc = B[CB_A_ST].ensure(na1 * 4)) || (rc = B[CB_A_LEN].ensure(na1 * 4)) ||
        (rc = B[CB_A_NC].ensure(na1 * 8)) || (rc = B[CB_A_BIN].ensure(na1 * 4)) ||
        (rc = B[CB_A_CB].ensure(na1 * 4)) || (rc = B[CB_A_CE].ensure(na1 * 4)) ||
        (rc = B[CB_A_SB].ensure(na1 * 4)) || (rc = B[CB_A_RPOS].ensure(na1 * 4)) ||
        (rc = B[CB_A_END].ensure(na1 * 4)) || (rc = B[CB_SORTED].ensure(na1 * 4)) ||
        (rc = B[CB_LST_SCORE].ensure(na1 * 8)) || (rc = B[CB_LST_ALN].ensure(na1 * 4)) ||
        (rc = B[CB_KEPT].ensure(na1)))
        return rc;
    if ((rc = B[CB_WORK].ensure(64))) return rc;
    if ((rc = B[CB_PROF].ensure(CNS_NPHASE * 8))) return rc;
    if ((rc = B[CB_RETRY].ensure(((size_t)n + 16) * 4))) return rc;
    if ((rc = upload(B[CB_OUT_OFF], c->out_off.data(), n + 1, s))) return rc;
    if ((rc = upload(B[CB_CHIM_OFF], c->chim_off.data(), n + 1, s))) return rc;
    const size_t n1 = (size_t)n + 1;
    if ((rc = B[CB_STATUS].ensure(n1 * 4)) || (rc = B[CB_SEQ_LEN].ensure(n1 * 4)) ||
        (rc = B[CB_TRACE_LEN].ensure(n1 * 4)) || (rc = B[CB_NCIGAR].ensure(n1 * 4)) ||
        (rc = B[CB_NCHIM].ensure(n1 * 4)))
        return rc;
    const size_t sc = (size_t)c->seq_cap + 1;
    if ((rc = B[CB_O_SEQ].ensure(sc)) || (rc = B[CB_O_QUAL].ensure(sc)) || (rc = B[CB_O_TRACE].ensure(sc)) ||
        (rc = B[CB_O_CIG].ensure(sc * 4)) || (rc = B[CB_O_CHIM].ensure(((size_t)c->chim_cap + 1) * 16)))
        return rc;
    HIPCHK(hipStreamSynchronize(s));
    c->cns_loaded = true;
    return 0;
}

extern "C" int pr_cns_launch(pr_ctx *c, const pr_cns_params *p) {
    if (!c || !p) return set_error(PR_ERR_ARG, "null arg");
    if (!c->cns_loaded) return set_error(PR_ERR_ARG, "no resident consensus batch (pr_cns_upload first)");
    if (p->qual_weighted)
        return set_error(PR_ERR_UNSUPPORTED, "--qual-weighted (ccseq/utg modes) is not implemented on the GPU path");
    if (!(p->bin_size >= 1.0)) return set_error(PR_ERR_ARG, "bin_size must be >= 1");
    HIPCHK(hipSetDevice(c->device));
    CnsParamsDev P;
    P.max_coverage = p->max_coverage;
    P.bin_size = p->bin_size;
    P.bin_max_bases = p->bin_size * p->max_coverage;   // Seq.pm:517
    P.indel_taboo = p->indel_taboo;
    P.trim = p->trim;
    P.indel_taboo_length = p->indel_taboo_length;
    P.min_aln_length = p->min_aln_length;
    P.max_ins_length = p->max_ins_length;
    P.fallback_phred = p->fallback_phred;
    P.phred_offset = p->phred_offset;
    P.ref_phred_offset = p->ref_phred_offset;
    P.use_ref_qual = p->use_ref_qual;
    P.detect_chimera = p->detect_chimera;
    P.invert_scores = p->invert_scores;
    DevBuf *B = c->cb;
    CnsDev D;
    std::memset(&D, 0, sizeof D);
    D.n_lr = c->n_lr;
    D.n_aln = c->n_aln;
    D.lr_off = B[CB_LR_OFF].as<int64_t>();
    D.ref_seq = c->has_ref ? B[CB_REF_SEQ].as<uint8_t>() : nullptr;
    D.ref_qual = c->has_qual ? B[CB_REF_QUAL].as<uint8_t>() : nullptr;
    D.ign_off = c->has_ign ? B[CB_IGN_OFF].as<int64_t>() : nullptr;
    D.ign = c->has_ign ? B[CB_IGN].as<int32_t>() : nullptr;
    D.aln_off = B[CB_ALN_OFF].as<int64_t>();
    D.pos = B[CB_POS].as<int32_t>();
    D.score = B[CB_SCORE].as<double>();
    D.aflags = B[CB_AFLAGS].as<uint8_t>();
    D.seq_off = B[CB_SEQ_OFF].as<int64_t>();
    D.lseq = B[CB_LSEQ].as<int32_t>();
    D.cig_off = B[CB_CIG_OFF].as<int64_t>();
    D.ncig = B[CB_NCIG].as<int32_t>();
    D.seq = B[CB_SEQ].as<uint8_t>();
    D.cig = B[CB_CIG].as<uint32_t>();
    D.a_st = B[CB_A_ST].as<uint32_t>();
    D.a_len = B[CB_A_LEN].as<int32_t>();
    D.a_nc = B[CB_A_NC].as<double>();
    D.a_bin = B[CB_A_BIN].as<int32_t>();
    D.a_cb = B[CB_A_CB].as<int32_t>();
    D.a_ce = B[CB_A_CE].as<int32_t>();
    D.a_sb = B[CB_A_SB].as<int32_t>();
    D.a_rpos = B[CB_A_RPOS].as<int32_t>();
    D.a_end = B[CB_A_END].as<int32_t>();
    D.sorted = B[CB_SORTED].as<int32_t>();
    D.lst_score = B[CB_LST_SCORE].as<double>();
    D.lst_aln = B[CB_LST_ALN].as<int32_t>();
    D.kept = B[CB_KEPT].as<uint8_t>();
    D.bin_off = B[CB_BIN_OFF].as<int64_t>();
    D.bin_bases = B[CB_BIN_BASES].as<int64_t>();
    D.work = B[CB_WORK].as<int32_t>();
    // per-phase clock counters (thread 0 reads the wall clock at every phase boundary): off by
    // default, PRGPU_CNS_PROF=1 turns them on (bench.py: one extra untimed step)
    {
        const char *pe = getenv("PRGPU_CNS_PROF");
        D.prof = (pe && atoi(pe) != 0) ? B[CB_PROF].as<unsigned long long>() : nullptr;
    }
    D.out_off = B[CB_OUT_OFF].as<int64_t>();
    D.chim_off = B[CB_CHIM_OFF].as<int64_t>();
    D.status = B[CB_STATUS].as<int32_t>();
    D.seq_len = B[CB_SEQ_LEN].as<int32_t>();
    D.trace_len = B[CB_TRACE_LEN].as<int32_t>();
    D.ncigar = B[CB_NCIGAR].as<int32_t>();
    D.nchim = B[CB_NCHIM].as<int32_t>();
    D.o_seq = B[CB_O_SEQ].as<uint8_t>();
    D.o_qual = B[CB_O_QUAL].as<uint8_t>();
    D.o_trace = B[CB_O_TRACE].as<uint8_t>();
    D.o_cig = B[CB_O_CIG].as<uint32_t>();
    D.o_chim = B[CB_O_CHIM].as<int32_t>();
    if (c->n_lr == 0) {
        c->cns_launched = true;
        return 0;
    }
    {
        // bins per read with this bin size (Seq.pm:1437-1444 _init_read_bins)
        const std::vector<int64_t> &lr = c->lr_off_host;
        c->bin_off.assign(c->n_lr + 1, 0);
        for (int i = 0; i < c->n_lr; ++i)
            c->bin_off[i + 1] = c->bin_off[i] + (int64_t)((double)(lr[i + 1] - lr[i]) / p->bin_size) + 1;
        int rc;
        if ((rc = upload(B[CB_BIN_OFF], c->bin_off.data(), c->n_lr + 1, c->stream))) return rc;
        if ((rc = B[CB_BIN_BASES].ensure((size_t)(c->bin_off[c->n_lr] + 1) * 8))) return rc;
        D.bin_off = B[CB_BIN_OFF].as<int64_t>();
        D.bin_bases = B[CB_BIN_BASES].as<int64_t>();
    }
    if (c->pipe && c->own) {
        // owned batch: short reads (nt4, global ids) from the task's pool, CIGARs in place in
        // the received wire pool, the ASCII consensus reference of the owned reads
        D.ref_seq = B[CB_REF_SEQ].as<uint8_t>();
        D.ref_nt4 = c->own_ref_nt4 ? 1 : 0;
        D.seq = c->own_sr_resident ? c->ls[c->ss_samp_off.empty() ? LS_SRSEQ : LS_SRSAMP].as<uint8_t>()
                                   : c->xb[XB_SR].as<uint8_t>();
        D.seq_nt4 = 1;
        D.cig = c->xb[XB_RCIG].as<uint32_t>();
        if (c->x_pass) {   // world 1: CIGARs in place in the SW output pool
            SwPtrs sp;
            int rc = sw_get_ptrs(c, &sp);
            if (rc) return rc;
            D.cig = sp.cig;
        }
    } else if (c->pipe) {
        // consensus reads the SW batch in place: long reads and short reads as
        // nt4, CIGARs in place in the SW output pool (per-task starts: pipe hand-off)
        SwPtrs sp;
        int rc = sw_get_ptrs(c, &sp);
        if (rc) return rc;
        if (c->pipe_ref_ascii) {   // bam2cns --ref differs from the mapping reference (masked HCRs)
            D.ref_seq = B[CB_REF_SEQ].as<uint8_t>();
            D.ref_nt4 = 0;
        } else {
            D.ref_seq = sp.lr;
            D.ref_nt4 = 1;
        }
        D.seq = sp.sr;
        D.seq_nt4 = 1;
        D.cig = sp.cig;
    }
    if (c->pipe && c->cns_gathered) {   // a second launch on the same hand-off: already in place
        D.seq = B[CB_SEQ].as<uint8_t>();
        D.cig = B[CB_CIG].as<uint32_t>();
    } else if (c->pipe && c->n_aln > 0 && !getenv("PRGPU_CNS_NOGATHER")) {
        // the alignments' SEQ bytes and CIGAR ops in consensus order (pipe_kernels.hip cns_gather):
        // into the standalone path's SEQ / CIGAR pools, which a pipe batch does not use
        const int64_t na = c->n_aln;
        const int64_t *tot = D.aln_off + c->n_lr;
        const size_t tb = cns_gather_temp_bytes(na);
        int rc;
        if ((rc = B[CB_GSZS].ensure((size_t)(na + 1) * 8)) || (rc = B[CB_GSZC].ensure((size_t)(na + 1) * 8)) ||
            (rc = B[CB_GSO].ensure((size_t)(na + 1) * 8)) || (rc = B[CB_GCO].ensure((size_t)(na + 1) * 8)) ||
            (rc = B[CB_GTMP].ensure(tb)))
            return rc;
        int e = cns_gather_offsets(tot, na, D.lseq, D.ncig, B[CB_GSZS].as<int64_t>(), B[CB_GSZC].as<int64_t>(),
                                   B[CB_GSO].as<int64_t>(), B[CB_GCO].as<int64_t>(), B[CB_GTMP].p, tb, (void *)c->stream);
        if (e) return set_error(PR_ERR_HIP, "consensus gather: %s", hipGetErrorString((hipError_t)e));
        int64_t tot_seq = 0, tot_cig = 0;
        HIPCHK(hipMemcpyAsync(&tot_seq, B[CB_GSO].as<int64_t>() + na, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(&tot_cig, B[CB_GCO].as<int64_t>() + na, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if ((rc = B[CB_SEQ].ensure((size_t)tot_seq + 16)) || (rc = B[CB_CIG].ensure((size_t)tot_cig * 4 + 16))) return rc;
        e = cns_gather_copy(tot, na, D.seq, D.cig, B[CB_SEQ_OFF].as<int64_t>(), D.lseq, B[CB_CIG_OFF].as<int64_t>(), D.ncig,
                            B[CB_GSO].as<int64_t>(),
                            B[CB_GCO].as<int64_t>(), B[CB_SEQ].as<uint8_t>(), B[CB_CIG].as<uint32_t>(), (void *)c->stream);
        if (e) return set_error(PR_ERR_HIP, "consensus gather: %s", hipGetErrorString((hipError_t)e));
        D.seq = B[CB_SEQ].as<uint8_t>();
        D.cig = B[CB_CIG].as<uint32_t>();
        c->cns_gathered = true;   // (the offsets now point into the gathered pools)
    }
    HIPCHK(hipMemsetAsync(D.work, 0, 64, c->stream));
    HIPCHK(hipMemsetAsync(B[CB_PROF].as<unsigned long long>(), 0, CNS_NPHASE * 8, c->stream));
    const int wgcu = cns_wg_per_cu();
    const int grid = c->n_lr < c->n_cu * wgcu ? c->n_lr : c->n_cu * wgcu;
    const int grid_retry = c->n_lr < c->n_cu ? c->n_lr : c->n_cu;
    {
        // K pool: per resident workgroup the window starts (longest read / 256 + 8 ints) and
        // 12 ints per kept alignment
        int64_t lmax = 0;
        for (int i = 0; i < c->n_lr; ++i) lmax = std::max(lmax, c->lr_off_host[i + 1] - c->lr_off_host[i]);
        const int64_t kc = ((lmax / 256 + 12) + 12 * (c->k_need < 64 ? 64 : c->k_need) + 3) & ~(int64_t)3;   // 16-byte entries
        int rc;
        if ((rc = B[CB_K].ensure((size_t)grid * kc * 4))) return rc;
        D.k_pool = B[CB_K].as<int32_t>();
        D.k_cap = kc;
        D.retry = B[CB_RETRY].as<int32_t>();
        D.retry_n = B[CB_RETRY].as<int32_t>() + c->n_lr + 8;
        HIPCHK(hipMemsetAsync(D.retry_n, 0, 4, c->stream));
        D.debug = getenv("PRGPU_CNS_DEBUG") ? atoi(getenv("PRGPU_CNS_DEBUG")) : 0;
        const char *fl = getenv("PRGPU_CNS_LARGE");   // diagnostics: all reads through the large geometry
        if (fl && atoi(fl)) {
            D.force_large = 1;
            std::vector<int32_t> all((size_t)c->n_lr + 1);
            for (int i = 0; i < c->n_lr; ++i) all[(size_t)i] = i;
            all[(size_t)c->n_lr] = c->n_lr;
            HIPCHK(hipMemcpyAsync(D.retry, all.data(), (size_t)c->n_lr * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(D.retry_n, &all[(size_t)c->n_lr], 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        }
    }
    HIPCHK(hipEventRecord(c->ev[4], c->stream));
    int e = cns_launch(D, P, grid, grid_retry, (void *)c->stream);
    if (e != 0) return set_error(PR_ERR_HIP, "cns kernel launch failed: %s", hipGetErrorString((hipError_t)e));
    HIPCHK(hipEventRecord(c->ev[5], c->stream));
    c->cns_launched = true;
    return 0;
}

template <class T>
static int download(T *h, const DevBuf &d, size_t n, hipStream_t s, size_t first = 0) {   // elements [first, first + n)
    if (h && n) HIPCHK(hipMemcpyAsync(h, d.as<T>() + first, n * sizeof(T), hipMemcpyDeviceToHost, s));
    return 0;
}

extern "C" int pr_cns_download(pr_ctx *c, pr_cns_out *o) {
    if (!c || !o) return set_error(PR_ERR_ARG, "null arg");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
    float ms = 0.f;
    if (c->n_lr && hipEventElapsedTime(&ms, c->ev[4], c->ev[5]) == hipSuccess) c->last_ms = ms;
    if (c->pipe && c->n_lr && hipEventElapsedTime(&ms, c->ev[0], c->ev[4]) == hipSuccess) c->ms_pipe = ms;
    const int n = c->n_lr;
    DevBuf *B = c->cb;
    int rc;
    if (o->out_off) std::memcpy(o->out_off, c->out_off.data(), (n + 1) * sizeof(int64_t));
    if (o->chim_off) std::memcpy(o->chim_off, c->chim_off.data(), (n + 1) * sizeof(int64_t));
    if ((rc = download(o->status, B[CB_STATUS], n, s)) || (rc = download(o->seq_len, B[CB_SEQ_LEN], n, s)) ||
        (rc = download(o->trace_len, B[CB_TRACE_LEN], n, s)) || (rc = download(o->ncigar, B[CB_NCIGAR], n, s)) ||
        (rc = download(o->nchim, B[CB_NCHIM], n, s)) || (rc = download(o->seq, B[CB_O_SEQ], c->seq_cap, s)) ||
        (rc = download(o->qual, B[CB_O_QUAL], c->seq_cap, s)) ||
        (rc = download(o->trace, B[CB_O_TRACE], c->seq_cap, s)) ||
        (rc = download(o->cigar, B[CB_O_CIG], c->seq_cap, s)) ||
        (rc = download(o->chim, B[CB_O_CHIM], c->chim_cap * 4, s)) ||
        (rc = download(o->kept, B[CB_KEPT], c->n_aln, s)))
        return rc;
    if (o->bin_bases && c->bin_off.size() == (size_t)n + 1)
        if ((rc = download(o->bin_bases, B[CB_BIN_BASES], c->bin_off[n], s))) return rc;
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

extern "C" int pr_cns_run(pr_ctx *c, const pr_cns_params *p, const pr_cns_batch *b, pr_cns_out *o) {
    int rc = pr_cns_upload(c, b);
    if (rc) return rc;
    if ((rc = pr_cns_launch(c, p))) return rc;
    return pr_cns_download(c, o);
}

extern "C" int pr_cns_last_timing(pr_ctx *c, double *ms_prep, double *ms_pileup) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    if (ms_prep) *ms_prep = 0.0;
    if (ms_pileup) *ms_pileup = c->last_ms;
    return 0;
}

extern "C" int pr_cns_phase_ticks(pr_ctx *c, uint64_t *ticks, int n) {
    if (!c || !ticks || n < 8) return set_error(PR_ERR_ARG, "need ctx and >= 8 ticks");
    if (!c->cns_loaded || !c->cb[CB_PROF].p) return set_error(PR_ERR_ARG, "no consensus launch yet");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(ticks, c->cb[CB_PROF].p, (size_t)(n < CNS_NPHASE ? n : CNS_NPHASE) * 8, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int pr_cns_resident_stats(pr_ctx *c, int64_t *columns, int64_t *alg_bytes) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    if (columns) *columns = c->total_cols;
    if (alg_bytes) *alg_bytes = c->alg_bytes;
    return 0;
}

// ---------------------------------------------------------------------------
// one iteration on the device: SW -> assemble -> consensus (pr_iter_*)
// dev_*: device sources in place of the batch's host pools (the resident long-read set and the
// seeding's copies: pr_iter_upload_lrset)
static int iter_upload(pr_ctx *c, const pr_iter_batch *b, bool gpu_seeds, const uint8_t *dev_sr = nullptr,
                       const uint8_t *dev_lr = nullptr, const uint8_t *dev_ref = nullptr,
                       const uint8_t *dev_qual = nullptr) {
    if (!c || !b) return set_error(PR_ERR_ARG, "null arg");
    pr_sw_batch sbv = b->sw;
    if (gpu_seeds) {   // the seeds of the last pr_seed_gpu_map, still in HBM
        if (c->seed_pre.size() != (size_t)sbv.n_sr + 1)
            return set_error(PR_ERR_ARG, "no device seeds for these short reads (pr_seed_gpu_map with out = NULL first)");
        sbv.n_task = c->seed_pre.back();
        sbv.t_sr = sbv.t_lr = sbv.t_qbeg = sbv.t_rbeg = sbv.t_slen = sbv.t_chain = nullptr;
        sbv.t_strand = nullptr;
    }
    const pr_sw_batch &sb = sbv;
    const int n = sb.n_lr;
    const bool bwa = sb.t_chain != nullptr || gpu_seeds;   // seeds in, alignments grouped by long read on the device
    if (!bwa && (!b->task_lr_off || b->task_lr_off[0] != 0 || b->task_lr_off[n] != sb.n_task))
        return set_error(PR_ERR_ARG, "task_lr_off must partition the tasks");
    int maxt = 1;
    for (int i = 0; i < n && !bwa; ++i) {
        if (b->task_lr_off[i + 1] < b->task_lr_off[i]) return set_error(PR_ERR_ARG, "task_lr_off not monotone");
        for (int64_t t = b->task_lr_off[i]; t < b->task_lr_off[i + 1]; ++t)
            if (sb.t_lr[t] != i) return set_error(PR_ERR_ARG, "tasks must be grouped by long read");
        const int64_t k = b->task_lr_off[i + 1] - b->task_lr_off[i];
        if (k > maxt) maxt = (int)k;
    }
    if (maxt > 16384) return set_error(PR_ERR_CAPACITY, "more than 16384 tasks on one long read");
    int rc = gpu_seeds ? sw_upload_device_seeds(c, &sb, c->sd[SB_DENSE].as<pr_seed_task>(), c->seed_pre.data(),
                                                dev_sr, dev_lr)
                       : pr_sw_upload(c, &sb);
    if (rc) return rc;
    c->x_ready = c->x_pass = false;   // a new SW batch: no exchange of it yet
    HIPCHK(hipSetDevice(c->device));
    c->cns_launched = false;
    c->iter_masked = false;
    c->own = false;
    hipStream_t s = c->stream;
    c->n_lr = n;
    c->n_aln = sb.n_task;
    c->total_cols = sb.lr_off[n];
    c->has_ref = true;
    c->pipe_ref_ascii = b->ref_seq != nullptr || dev_ref != nullptr;
    c->has_qual = b->lr_qual != nullptr || dev_qual != nullptr;
    c->has_ign = false;
    c->lr_off_host.assign(sb.lr_off, sb.lr_off + n + 1);
    c->out_off.assign(n + 1, 0);
    c->chim_off.assign(n + 1, 0);
    for (int i = 0; i < n; ++i) {
        const int64_t L = sb.lr_off[i + 1] - sb.lr_off[i];
        const int64_t nb = (int64_t)((double)L / 20.0) + 1;
        c->out_off[i + 1] = c->out_off[i] + 2 * L + 1024;   // guarded in the kernel
        c->chim_off[i + 1] = c->chim_off[i] + nb / 2 + 2;
    }
    c->seq_cap = c->out_off[n];
    c->chim_cap = c->chim_off[n];
    c->alg_bytes = 0;
    c->k_need = maxt;
    int sc = 1;
    while (sc < maxt) sc <<= 1;
    c->pipe_sort_cap = sc;
    DevBuf *B = c->cb;
    const size_t na1 = (size_t)sb.n_task + 1, n1 = (size_t)n + 1;
    if ((rc = upload(B[CB_LR_OFF], sb.lr_off, n1, s))) return rc;
    if (b->lr_qual && (rc = upload(B[CB_REF_QUAL], b->lr_qual, (size_t)sb.lr_off[n], s))) return rc;
    if (b->ref_seq && (rc = upload(B[CB_REF_SEQ], b->ref_seq, (size_t)sb.lr_off[n], s))) return rc;
    for (int k = 0; k < 2; ++k) {   // device sources of the reference and its qualities
        const uint8_t *src = k ? dev_qual : dev_ref;
        if (!src) continue;
        DevBuf &dst = B[k ? CB_REF_QUAL : CB_REF_SEQ];
        if ((rc = dst.ensure((size_t)sb.lr_off[n] + 1))) return rc;
        if (sb.lr_off[n]) HIPCHK(hipMemcpyAsync(dst.p, src, (size_t)sb.lr_off[n], hipMemcpyDeviceToDevice, s));
    }
    if (!bwa && (rc = upload(c->pb[0], b->task_lr_off, n1, s))) return rc;
    if ((rc = c->pb[1].ensure(n1 * 4)) || (rc = c->pb[2].ensure(n1 * 4))) return rc;
    if ((rc = B[CB_ALN_OFF].ensure(n1 * 8)) || (rc = B[CB_POS].ensure(na1 * 4)) ||
        (rc = B[CB_SCORE].ensure(na1 * 8)) || (rc = B[CB_AFLAGS].ensure(na1)) ||
        (rc = B[CB_SEQ_OFF].ensure(na1 * 8)) || (rc = B[CB_LSEQ].ensure(na1 * 4)) ||
        (rc = B[CB_CIG_OFF].ensure(na1 * 8)) || (rc = B[CB_NCIG].ensure(na1 * 4)))
        return rc;
    if ((rc = B[CB_A_ST].ensure(na1 * 4)) || (rc = B[CB_A_LEN].ensure(na1 * 4)) ||
        (rc = B[CB_A_NC].ensure(na1 * 8)) || (rc = B[CB_A_BIN].ensure(na1 * 4)) ||
        (rc = B[CB_A_CB].ensure(na1 * 4)) || (rc = B[CB_A_CE].ensure(na1 * 4)) ||
        (rc = B[CB_A_SB].ensure(na1 * 4)) || (rc = B[CB_A_RPOS].ensure(na1 * 4)) ||
        (rc = B[CB_A_END].ensure(na1 * 4)) || (rc = B[CB_SORTED].ensure(na1 * 4)) ||
        (rc = B[CB_LST_SCORE].ensure(na1 * 8)) || (rc = B[CB_LST_ALN].ensure(na1 * 4)) ||
        (rc = B[CB_KEPT].ensure(na1)) || (rc = B[CB_WORK].ensure(64)) ||
        (rc = B[CB_PROF].ensure(CNS_NPHASE * 8)) || (rc = B[CB_RETRY].ensure(((size_t)n + 16) * 4)))
        return rc;
    if ((rc = upload(B[CB_OUT_OFF], c->out_off.data(), n1, s))) return rc;
    if ((rc = upload(B[CB_CHIM_OFF], c->chim_off.data(), n1, s))) return rc;
    if ((rc = B[CB_STATUS].ensure(n1 * 4)) || (rc = B[CB_SEQ_LEN].ensure(n1 * 4)) ||
        (rc = B[CB_TRACE_LEN].ensure(n1 * 4)) || (rc = B[CB_NCIGAR].ensure(n1 * 4)) ||
        (rc = B[CB_NCHIM].ensure(n1 * 4)))
        return rc;
    const size_t scap = (size_t)c->seq_cap + 1;
    if ((rc = B[CB_O_SEQ].ensure(scap)) || (rc = B[CB_O_QUAL].ensure(scap)) || (rc = B[CB_O_TRACE].ensure(scap)) ||
        (rc = B[CB_O_CIG].ensure(scap * 4)) || (rc = B[CB_O_CHIM].ensure(((size_t)c->chim_cap + 1) * 16)))
        return rc;
    HIPCHK(hipStreamSynchronize(s));
    c->cns_loaded = true;
    c->pipe = true;
    return 0;
}

extern "C" int pr_iter_upload(pr_ctx *c, const pr_iter_batch *b) { return iter_upload(c, b, false); }
extern "C" int pr_iter_upload_gpu_seeds(pr_ctx *c, const pr_iter_batch *b) { return iter_upload(c, b, true); }

// ---------------------------------------------------------------------------
// exact-parity multi-GPU layout (include/prgpu.h: pr_sw_upload_gpu_seeds, pr_aln_exchange,
// pr_iter_upload_owned, then pr_iter_launch on the owned batch)
extern "C" int pr_sw_upload_gpu_seeds(pr_ctx *c, const pr_sw_batch *b) {
    if (!c || !b) return set_error(PR_ERR_ARG, "null arg");
    if (c->seed_pre.size() != (size_t)b->n_sr + 1)
        return set_error(PR_ERR_ARG, "no device seeds for these short reads (pr_seed_gpu_map with out = NULL first)");
    pr_sw_batch sb = *b;
    sb.n_task = c->seed_pre.back();
    sb.t_sr = sb.t_lr = sb.t_qbeg = sb.t_rbeg = sb.t_slen = sb.t_chain = nullptr;
    sb.t_strand = nullptr;
    // pools left NULL: the device copies the seeding made (no second host upload)
    const uint8_t *dsr = nullptr, *dlr = nullptr;
    if (!b->sr_seq) {
        if (b->n_sr && c->seed_sr_bases != b->sr_off[b->n_sr])
            return set_error(PR_ERR_ARG, "sr_seq NULL: the short reads must be those of the last pr_seed_gpu_map");
        dsr = c->sd[SB_SEQ].as<uint8_t>();
    }
    if (!b->lr_seq) {
        if (!c->seed_n_text || c->seed_view.l_pac != b->lr_off[b->n_lr] || c->seed_view.n_lr != b->n_lr)
            return set_error(PR_ERR_ARG, "lr_seq NULL: the long reads must be those of the last pr_seed_gpu_index_build");
        dlr = c->sd[SX_LRSEQ].as<uint8_t>();
    }
    c->x_ready = c->x_pass = false;   // a new SW batch: no exchange of it yet
    const int rc = sw_upload_device_seeds(c, &sb, c->sd[SB_DENSE].as<pr_seed_task>(), c->seed_pre.data(), dsr, dlr);
    // the seeding's short-read pool is handed over once: a later batch with the same base count
    // (another sample, another shard) must not pick it up silently (the next map sets it again)
    if (!rc && dsr) c->seed_sr_bases = -1;
    return rc;
}

// the sender half of the exchange: the reported alignments of the last bwa-mode pr_sw_launch
// packed by owner into XB_SREC / XB_SCIG; counts (records, ops) per owner into cnt (syncs)
static int xchg_pack(pr_ctx *c, int world, int64_t sr0, const int64_t *lr_bounds, std::vector<int64_t> &n_rec,
                     std::vector<int64_t> &n_ops) {
    if (world < 1 || world > 64) return set_error(PR_ERR_CAPACITY, "1 to 64 ranks");
    if (lr_bounds[0] != 0) return set_error(PR_ERR_ARG, "lr_bounds must start at 0");
    for (int r = 0; r < world; ++r)
        if (lr_bounds[r + 1] < lr_bounds[r]) return set_error(PR_ERR_ARG, "lr_bounds must be ascending");
    XchgSend X;
    std::memset(&X, 0, sizeof X);
    int rc;
    if ((rc = sw_xchg_send(c, &X))) return rc;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    DevBuf *B = c->xb;
    const size_t n1 = (size_t)X.n + 1;
    if ((rc = upload(B[XB_BOUNDS], lr_bounds, (size_t)world + 1, s)) || (rc = B[XB_KEY0].ensure(n1 * 4)) ||
        (rc = B[XB_KEY1].ensure(n1 * 4)) || (rc = B[XB_IDX0].ensure(n1 * 4)) || (rc = B[XB_IDX1].ensure(n1 * 4)) ||
        (rc = B[XB_CNT].ensure(2 * 65 * 8)) || (rc = B[XB_OPIN].ensure(n1 * 8)) || (rc = B[XB_OPAT].ensure(n1 * 8)) ||
        (rc = B[XB_SREC].ensure(n1 * sizeof(XRec))))
        return rc;
    const size_t tb = xchg_temp_bytes(X.n, 1);
    if ((rc = B[XB_TEMP].ensure(tb))) return rc;
    X.bounds = B[XB_BOUNDS].as<int64_t>();
    X.world = world;
    X.sr0 = sr0;
    X.key0 = B[XB_KEY0].as<int32_t>();
    X.key1 = B[XB_KEY1].as<int32_t>();
    X.idx0 = B[XB_IDX0].as<int32_t>();
    X.idx1 = B[XB_IDX1].as<int32_t>();
    X.cnt = B[XB_CNT].as<unsigned long long>();
    X.op_in = B[XB_OPIN].as<int64_t>();
    X.op_at = B[XB_OPAT].as<int64_t>();
    X.rec = B[XB_SREC].as<XRec>();
    int e = xchg_pack_launch(X, B[XB_TEMP].p, B[XB_TEMP].cap, (void *)s);
    if (e) return set_error(PR_ERR_HIP, "exchange pack: %s", hipGetErrorString((hipError_t)e));
    std::vector<unsigned long long> cnt((size_t)2 * (world + 1), 0ull);
    HIPCHK(hipMemcpyAsync(cnt.data(), X.cnt, cnt.size() * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    n_rec.assign((size_t)world, 0);
    n_ops.assign((size_t)world, 0);
    int64_t ops = 0;
    for (int r = 0; r < world; ++r) {
        n_rec[(size_t)r] = (int64_t)cnt[(size_t)r];
        n_ops[(size_t)r] = (int64_t)cnt[(size_t)world + 1 + r];
        ops += n_ops[(size_t)r];
    }
    if ((rc = B[XB_SCIG].ensure(((size_t)ops + 1) * 4))) return rc;
    X.wcig = B[XB_SCIG].as<uint32_t>();
    if ((e = xchg_write_launch(X, (void *)s))) return set_error(PR_ERR_HIP, "exchange pack: %s", hipGetErrorString((hipError_t)e));
    return 0;
}

static int xchg_recv_buffers(pr_ctx *c, int64_t rec_bytes, int64_t cig_bytes) {
    if (rec_bytes % (int64_t)sizeof(XRec)) return set_error(PR_ERR_ARG, "exchange: ragged record counts");
    c->x_nrecv = rec_bytes / (int64_t)sizeof(XRec);
    c->x_nrcig = cig_bytes / 4;
    int rc;
    if ((rc = c->xb[XB_RREC].ensure((size_t)rec_bytes + sizeof(XRec))) || (rc = c->xb[XB_RCIG].ensure((size_t)cig_bytes + 64)))
        return rc;
    return 0;
}

extern "C" int pr_aln_exchange(pr_ctx *c, pr_comm *comm, int64_t sr0, const int64_t *lr_bounds, int64_t *n_recv) {
    if (!c || !lr_bounds) return set_error(PR_ERR_ARG, "null arg");
    int rank = 0, world = 1, rc;
    if (comm) {
        if (comm_ctx(comm) != c) return set_error(PR_ERR_ARG, "the communicator belongs to another context");
        if ((rc = pr_comm_rank(comm, &rank, &world))) return rc;
    }
    c->x_ready = false;
    c->x_pass = false;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventRecord(c->ev[0], c->stream));   // pr_iter_last_timing: the hand-off includes the exchange
    if (world == 1 && sr0 == 0 && !getenv("PRGPU_XCHG_FORCE")) {
        // one rank holding every short read: it owns every long read, nothing moves -- the owned
        // launch takes the SW output directly (PRGPU_XCHG_FORCE=1: pack and copy anyway, a test hook)
        XchgSend X;
        if ((rc = sw_xchg_send(c, &X))) return rc;
        c->x_pass = true;
        c->x_ready = true;
        c->x_nrecv = X.n;
        c->x_from.assign(1, X.n);
        if (n_recv) *n_recv = X.n;
        return 0;
    }
    std::vector<int64_t> nrec, nops;
    rc = xchg_pack(c, world, sr0, lr_bounds, nrec, nops);
    // the pack is local: every rank learns whether all packed before any data moves
    if (comm) rc = pr_comm_agree(comm, rc);
    if (rc) return rc;
    std::vector<int64_t> sc_rec((size_t)world), sc_cig((size_t)world), rc_rec((size_t)world), rc_cig((size_t)world);
    for (int r = 0; r < world; ++r) {
        sc_rec[(size_t)r] = nrec[(size_t)r] * (int64_t)sizeof(XRec);
        sc_cig[(size_t)r] = nops[(size_t)r] * 4;
    }
    if (comm) {
        if ((rc = pr_comm_alltoall_counts(comm, sc_rec.data(), rc_rec.data())) ||
            (rc = pr_comm_alltoall_counts(comm, sc_cig.data(), rc_cig.data())))
            return rc;
    } else {
        rc_rec = sc_rec;
        rc_cig = sc_cig;
    }
    int64_t nr = 0, nc = 0;
    c->x_from.assign((size_t)world, 0);
    for (int r = 0; r < world; ++r) {
        nr += rc_rec[(size_t)r];
        nc += rc_cig[(size_t)r];
        c->x_from[(size_t)r] = rc_rec[(size_t)r] / (int64_t)sizeof(XRec);
    }
    rc = xchg_recv_buffers(c, nr, nc);
    // the receive buffers are a local allocation: a rank that could not get them must not leave
    // the others inside the all-to-all
    if (comm) rc = pr_comm_agree(comm, rc);
    if (rc) return rc;
    DevBuf *B = c->xb;
    if (comm) {
        if ((rc = pr_comm_alltoallv_dev(comm, B[XB_SREC].p, sc_rec.data(), B[XB_RREC].p, rc_rec.data())) ||
            (rc = pr_comm_alltoallv_dev(comm, B[XB_SCIG].p, sc_cig.data(), B[XB_RCIG].p, rc_cig.data())))
            return rc;
    } else {
        HIPCHK(hipSetDevice(c->device));
        if (nr) HIPCHK(hipMemcpyAsync(B[XB_RREC].p, B[XB_SREC].p, (size_t)nr, hipMemcpyDeviceToDevice, c->stream));
        if (nc) HIPCHK(hipMemcpyAsync(B[XB_RCIG].p, B[XB_SCIG].p, (size_t)nc, hipMemcpyDeviceToDevice, c->stream));
    }
    c->x_ready = true;
    if (n_recv) *n_recv = c->x_nrecv;
    return 0;
}

extern "C" int pr_aln_exchange_local(pr_ctx *const *ctxs, int world, const int64_t *sr0, const int64_t *lr_bounds,
                                     int64_t *n_recv) {
    // the same exchange among `world` contexts of one process (e.g. several shards on one GPU):
    // the packs, then device-to-device block copies in source order instead of RCCL
    if (!ctxs || !sr0 || !lr_bounds || world < 1) return set_error(PR_ERR_ARG, "bad arg");
    std::vector<std::vector<int64_t>> nrec((size_t)world), nops((size_t)world);
    int rc;
    for (int k = 0; k < world; ++k) {
        if (!ctxs[k]) return set_error(PR_ERR_ARG, "null context");
        ctxs[k]->x_ready = false;
        ctxs[k]->x_pass = false;   // the owned launch reads the records copied below
        if ((rc = xchg_pack(ctxs[k], world, sr0[k], lr_bounds, nrec[(size_t)k], nops[(size_t)k]))) return rc;
    }
    for (int k = 0; k < world; ++k) {
        HIPCHK(hipSetDevice(ctxs[k]->device));
        HIPCHK(hipStreamSynchronize(ctxs[k]->stream));
    }
    for (int r = 0; r < world; ++r) {
        pr_ctx *d = ctxs[r];
        int64_t nr = 0, nc = 0;
        d->x_from.assign((size_t)world, 0);
        for (int k = 0; k < world; ++k) {
            nr += nrec[(size_t)k][(size_t)r] * (int64_t)sizeof(XRec);
            nc += nops[(size_t)k][(size_t)r] * 4;
            d->x_from[(size_t)k] = nrec[(size_t)k][(size_t)r];
        }
        if ((rc = xchg_recv_buffers(d, nr, nc))) return rc;
        int64_t ro = 0, co = 0;
        for (int k = 0; k < world; ++k) {
            int64_t so = 0, sco = 0;   // this destination's block in the source's send buffers
            for (int q = 0; q < r; ++q) {
                so += nrec[(size_t)k][(size_t)q] * (int64_t)sizeof(XRec);
                sco += nops[(size_t)k][(size_t)q] * 4;
            }
            const int64_t bn = nrec[(size_t)k][(size_t)r] * (int64_t)sizeof(XRec), bc = nops[(size_t)k][(size_t)r] * 4;
            HIPCHK(hipSetDevice(d->device));
            if (bn) HIPCHK(hipMemcpyAsync((uint8_t *)d->xb[XB_RREC].p + ro, (uint8_t *)ctxs[k]->xb[XB_SREC].p + so,
                                          (size_t)bn, hipMemcpyDeviceToDevice, d->stream));
            if (bc) HIPCHK(hipMemcpyAsync((uint8_t *)d->xb[XB_RCIG].p + co, (uint8_t *)ctxs[k]->xb[XB_SCIG].p + sco,
                                          (size_t)bc, hipMemcpyDeviceToDevice, d->stream));
            ro += bn;
            co += bc;
        }
        HIPCHK(hipStreamSynchronize(d->stream));
        d->x_ready = true;
        if (n_recv) n_recv[r] = d->x_nrecv;
    }
    return 0;
}

extern "C" int pr_aln_exchange_sources(pr_ctx *c, int64_t *per_rank, int cap, int *world) {
    if (!c || (cap && !per_rank)) return set_error(PR_ERR_ARG, "null arg");
    if (!c->x_ready) return set_error(PR_ERR_ARG, "no exchange yet");
    for (int r = 0; r < cap && r < (int)c->x_from.size(); ++r) per_rank[r] = c->x_from[(size_t)r];
    if (world) *world = (int)c->x_from.size();
    return 0;
}

extern "C" int pr_iter_upload_owned(pr_ctx *c, const pr_own_batch *b) {
    if (!c || !b) return set_error(PR_ERR_ARG, "null arg");
    const int n = b->n_lr;
    if (n < 0 || b->n_sr < 0 || (n && !b->lr_off) || !b->sr_off)
        return set_error(PR_ERR_ARG, "owned batch: lr_off and the short-read offsets are required");
    if (n && b->lr_off[0] != 0) return set_error(PR_ERR_ARG, "lr_off must start at 0");
    for (int i = 0; i < n; ++i)
        if (b->lr_off[i + 1] < b->lr_off[i]) return set_error(PR_ERR_ARG, "lr_off not monotone");
    for (int i = 0; i < b->n_sr; ++i)
        if (b->sr_off[i + 1] < b->sr_off[i]) return set_error(PR_ERR_ARG, "sr_off not monotone");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    c->cns_launched = false;
    c->iter_masked = false;
    c->n_lr = n;
    c->n_aln = 0;   // the received alignments (sized at launch: own_group)
    const int64_t tl = n ? b->lr_off[n] : 0;
    c->total_cols = tl;
    c->has_ref = true;
    c->pipe_ref_ascii = true;
    const bool from_set = (b->from_set & PR_OWN_FROM_SET) != 0, sr_res = (b->from_set & PR_OWN_RESIDENT_SR) != 0;
    c->has_qual = b->lr_qual != nullptr || from_set;
    c->has_ign = false;
    c->lr_off_host.assign(b->lr_off, b->lr_off + n + 1);
    if (!n) c->lr_off_host.assign(1, 0);
    c->out_off.assign(n + 1, 0);
    c->chim_off.assign(n + 1, 0);
    for (int i = 0; i < n; ++i) {
        const int64_t L = b->lr_off[i + 1] - b->lr_off[i];
        const int64_t nb = (int64_t)((double)L / 20.0) + 1;
        c->out_off[i + 1] = c->out_off[i] + 2 * L + 1024;   // guarded in the kernel
        c->chim_off[i + 1] = c->chim_off[i] + nb / 2 + 2;
    }
    int64_t set0 = 0;   // from_set: the owned reads' first base in the set
    if (from_set) {
        if (c->ls_n < 0) return set_error(PR_ERR_ARG, "from_set: no resident long-read set");
        if (b->lr0 < 0 || b->lr0 + n > c->ls_n) return set_error(PR_ERR_ARG, "owned long reads outside the set");
        set0 = c->ls_off[(size_t)b->lr0];
        for (int i = 0; i <= n; ++i)
            if (c->ls_off[(size_t)(b->lr0 + i)] - set0 != b->lr_off[i])
                return set_error(PR_ERR_ARG, "owned long reads differ from the set's");
    }
    c->seq_cap = c->out_off[n];
    c->chim_cap = c->chim_off[n];
    c->alg_bytes = 0;
    c->k_need = 1;
    c->pipe_sort_cap = 1;
    DevBuf *B = c->cb;
    const size_t n1 = (size_t)n + 1;
    if ((rc = upload(B[CB_LR_OFF], c->lr_off_host.data(), n1, s))) return rc;
    if (!from_set && b->lr_qual && (rc = upload(B[CB_REF_QUAL], b->lr_qual, (size_t)tl, s))) return rc;
    // ref_seq / sr_seq NULL: the resident SW batch's long reads (the owned slice, nt4: the mapping
    // reference is the consensus reference) / short reads (every short read of the task) on the device
    SwPtrs sp{};
    if (((!b->ref_seq && !from_set) || (!b->sr_seq && !sr_res)) && (rc = sw_get_ptrs(c, &sp))) return rc;
    c->own_ref_nt4 = !b->ref_seq && !from_set;
    if (from_set) {   // the set's reads and qualities (the previous task's consensus)
        if ((rc = B[CB_REF_SEQ].ensure((size_t)tl + 1)) || (rc = B[CB_REF_QUAL].ensure((size_t)tl + 1))) return rc;
        if (tl) {
            HIPCHK(hipMemcpyAsync(B[CB_REF_SEQ].p, c->ls[LS_SEQ].as<uint8_t>() + set0, (size_t)tl, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(B[CB_REF_QUAL].p, c->ls[LS_QUAL].as<uint8_t>() + set0, (size_t)tl, hipMemcpyDeviceToDevice, s));
        }
    } else if (b->ref_seq) {
        if ((rc = upload(B[CB_REF_SEQ], b->ref_seq, (size_t)tl, s))) return rc;
    } else {
        if (b->lr0 < 0 || b->lr0 + n > sp.n_lr) return set_error(PR_ERR_ARG, "owned long reads outside the SW batch");
        int64_t base = 0, end = 0;
        HIPCHK(hipMemcpyAsync(&base, sp.lr_off + b->lr0, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&end, sp.lr_off + b->lr0 + n, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (end - base != tl) return set_error(PR_ERR_ARG, "owned long reads differ from the SW batch's");
        if ((rc = B[CB_REF_SEQ].ensure((size_t)tl + 1))) return rc;
        if (tl) HIPCHK(hipMemcpyAsync(B[CB_REF_SEQ].p, sp.lr + base, (size_t)tl, hipMemcpyDeviceToDevice, s));
    }
    if ((rc = upload(c->xb[XB_SROFF], b->sr_off, (size_t)b->n_sr + 1, s))) return rc;
    c->own_sr_resident = sr_res;
    if (sr_res) {   // the resident short reads (pr_srset_load, or the task sample) are the task's: read in place
        if (b->sr_seq) return set_error(PR_ERR_ARG, "PR_OWN_RESIDENT_SR: sr_seq must be NULL");
        const std::vector<int64_t> &ro = c->ss_samp_off.empty() ? c->ss_off : c->ss_samp_off;
        // every offset, not only the count and total: a batch with another per-read layout of the
        // same size would read the wrong bases
        if (ro.size() != (size_t)b->n_sr + 1 || !std::equal(ro.begin(), ro.end(), b->sr_off))
            return set_error(PR_ERR_ARG, "PR_OWN_RESIDENT_SR: sr_off differs from the resident short reads (pr_srset_load / "
                                         "pr_srset_sample)");
    } else if (b->sr_seq) {
        if ((rc = upload(c->xb[XB_SR], b->sr_seq, (size_t)b->sr_off[b->n_sr], s))) return rc;
    } else {
        if (sp.n_sr != b->n_sr) return set_error(PR_ERR_ARG, "sr_seq NULL: the SW batch must hold every short read");
        if ((rc = c->xb[XB_SR].ensure((size_t)b->sr_off[b->n_sr] + 1))) return rc;
        if (b->sr_off[b->n_sr])
            HIPCHK(hipMemcpyAsync(c->xb[XB_SR].p, sp.sr, (size_t)b->sr_off[b->n_sr], hipMemcpyDeviceToDevice, s));
    }
    if ((rc = c->pb[1].ensure(n1 * 4)) || (rc = c->pb[2].ensure(n1 * 4))) return rc;
    if ((rc = B[CB_ALN_OFF].ensure(n1 * 8)) || (rc = B[CB_WORK].ensure(64)) || (rc = B[CB_PROF].ensure(CNS_NPHASE * 8)) ||
        (rc = B[CB_RETRY].ensure(((size_t)n + 16) * 4)))
        return rc;
    if ((rc = upload(B[CB_OUT_OFF], c->out_off.data(), n1, s))) return rc;
    if ((rc = upload(B[CB_CHIM_OFF], c->chim_off.data(), n1, s))) return rc;
    if ((rc = B[CB_STATUS].ensure(n1 * 4)) || (rc = B[CB_SEQ_LEN].ensure(n1 * 4)) ||
        (rc = B[CB_TRACE_LEN].ensure(n1 * 4)) || (rc = B[CB_NCIGAR].ensure(n1 * 4)) ||
        (rc = B[CB_NCHIM].ensure(n1 * 4)))
        return rc;
    const size_t scap = (size_t)c->seq_cap + 1;
    if ((rc = B[CB_O_SEQ].ensure(scap)) || (rc = B[CB_O_QUAL].ensure(scap)) || (rc = B[CB_O_TRACE].ensure(scap)) ||
        (rc = B[CB_O_CIG].ensure(scap * 4)) || (rc = B[CB_O_CHIM].ensure(((size_t)c->chim_cap + 1) * 16)))
        return rc;
    DevBuf *X = c->xb;
    if ((rc = X[XB_GCNT].ensure(n1 * 4)) || (rc = X[XB_GCNT64].ensure(n1 * 8)) || (rc = X[XB_TASKOFF].ensure(n1 * 8)) ||
        (rc = X[XB_ERR].ensure(16)))
        return rc;
    HIPCHK(hipStreamSynchronize(s));
    c->own_lr0 = b->lr0;
    c->own = true;
    c->cns_loaded = true;
    c->pipe = true;
    return 0;
}

// owned batch: the received records regrouped by long read into the hand-off's inputs
static int own_group(pr_ctx *c, SwPtrs *sp) {
    if (!c->x_ready) return set_error(PR_ERR_ARG, "no received alignments (pr_aln_exchange first)");
    hipStream_t s = c->stream;
    DevBuf *B = c->xb;
    if (c->x_pass) {   // world 1: the SW output regrouped by long read, as pr_iter_launch does
        int rc = sw_get_pipe_ptrs(c, sp, true);
        if (rc) return rc;
        c->n_aln = sp->n_task;
        const size_t na1 = (size_t)sp->n_task + 1;
        DevBuf *C = c->cb;
        if ((rc = C[CB_POS].ensure(na1 * 4)) || (rc = C[CB_SCORE].ensure(na1 * 8)) || (rc = C[CB_AFLAGS].ensure(na1)) ||
            (rc = C[CB_SEQ_OFF].ensure(na1 * 8)) || (rc = C[CB_LSEQ].ensure(na1 * 4)) ||
            (rc = C[CB_CIG_OFF].ensure(na1 * 8)) || (rc = C[CB_NCIG].ensure(na1 * 4)) ||
            (rc = C[CB_A_ST].ensure(na1 * 4)) || (rc = C[CB_A_LEN].ensure(na1 * 4)) ||
            (rc = C[CB_A_NC].ensure(na1 * 8)) || (rc = C[CB_A_BIN].ensure(na1 * 4)) ||
            (rc = C[CB_A_CB].ensure(na1 * 4)) || (rc = C[CB_A_CE].ensure(na1 * 4)) ||
            (rc = C[CB_A_SB].ensure(na1 * 4)) || (rc = C[CB_A_RPOS].ensure(na1 * 4)) ||
            (rc = C[CB_A_END].ensure(na1 * 4)) || (rc = C[CB_SORTED].ensure(na1 * 4)) ||
            (rc = C[CB_LST_SCORE].ensure(na1 * 8)) || (rc = C[CB_LST_ALN].ensure(na1 * 4)) || (rc = C[CB_KEPT].ensure(na1)))
            return rc;
        return 0;
    }
    {   // per-alignment arrays of the hand-off and the consensus, sized by what arrived
        c->n_aln = c->x_nrecv;
        const size_t na1 = (size_t)c->x_nrecv + 1;
        DevBuf *C = c->cb;
        int rc;
        if ((rc = C[CB_POS].ensure(na1 * 4)) || (rc = C[CB_SCORE].ensure(na1 * 8)) || (rc = C[CB_AFLAGS].ensure(na1)) ||
            (rc = C[CB_SEQ_OFF].ensure(na1 * 8)) || (rc = C[CB_LSEQ].ensure(na1 * 4)) ||
            (rc = C[CB_CIG_OFF].ensure(na1 * 8)) || (rc = C[CB_NCIG].ensure(na1 * 4)) ||
            (rc = C[CB_A_ST].ensure(na1 * 4)) || (rc = C[CB_A_LEN].ensure(na1 * 4)) ||
            (rc = C[CB_A_NC].ensure(na1 * 8)) || (rc = C[CB_A_BIN].ensure(na1 * 4)) ||
            (rc = C[CB_A_CB].ensure(na1 * 4)) || (rc = C[CB_A_CE].ensure(na1 * 4)) ||
            (rc = C[CB_A_SB].ensure(na1 * 4)) || (rc = C[CB_A_RPOS].ensure(na1 * 4)) ||
            (rc = C[CB_A_END].ensure(na1 * 4)) || (rc = C[CB_SORTED].ensure(na1 * 4)) ||
            (rc = C[CB_LST_SCORE].ensure(na1 * 8)) || (rc = C[CB_LST_ALN].ensure(na1 * 4)) ||
            (rc = C[CB_KEPT].ensure(na1)) || (rc = B[XB_RCIGAT].ensure(na1 * 8)) || (rc = B[XB_GSR].ensure(na1 * 4)) ||
            (rc = B[XB_GSTATUS].ensure(na1 * 4)) || (rc = B[XB_GPOS].ensure(na1 * 4)) ||
            (rc = B[XB_GSCORE].ensure(na1 * 4)) || (rc = B[XB_GNCIG].ensure(na1 * 4)) ||
            (rc = B[XB_GCIGAT].ensure(na1 * 8)) || (rc = B[XB_GSTRAND].ensure(na1)) || (rc = B[XB_GPASS].ensure(na1)) ||
            (rc = B[XB_KEY0].ensure(na1 * 4)) || (rc = B[XB_KEY1].ensure(na1 * 4)) || (rc = B[XB_IDX0].ensure(na1 * 4)) ||
            (rc = B[XB_IDX1].ensure(na1 * 4)) || (rc = B[XB_OPIN].ensure(na1 * 8)))
            return rc;
        const size_t tb = xchg_temp_bytes(c->x_nrecv, c->n_lr);
        if ((rc = B[XB_TEMP].ensure(tb))) return rc;
    }
    XchgRecv R;
    std::memset(&R, 0, sizeof R);
    R.n = c->x_nrecv;
    R.rec = B[XB_RREC].as<XRec>();
    R.lr0 = c->own_lr0;
    R.n_lr = c->n_lr;
    R.key0 = B[XB_KEY0].as<int32_t>();
    R.key1 = B[XB_KEY1].as<int32_t>();
    R.idx0 = B[XB_IDX0].as<int32_t>();
    R.idx1 = B[XB_IDX1].as<int32_t>();
    R.cnt = B[XB_GCNT].as<int32_t>();
    R.cnt64 = B[XB_GCNT64].as<int64_t>();
    R.task_off = B[XB_TASKOFF].as<int64_t>();
    R.op_in = B[XB_OPIN].as<int64_t>();
    R.rcig_at = B[XB_RCIGAT].as<int64_t>();
    R.err = B[XB_ERR].as<int32_t>();
    R.o_sr = B[XB_GSR].as<int32_t>();
    R.o_status = B[XB_GSTATUS].as<int32_t>();
    R.o_pos = B[XB_GPOS].as<int32_t>();
    R.o_score = B[XB_GSCORE].as<int32_t>();
    R.o_ncig = B[XB_GNCIG].as<int32_t>();
    R.o_cig_at = B[XB_GCIGAT].as<int64_t>();
    R.o_strand = B[XB_GSTRAND].as<uint8_t>();
    R.o_pass = B[XB_GPASS].as<uint8_t>();
    int e = xchg_group_launch(R, B[XB_TEMP].p, B[XB_TEMP].cap, (void *)s);
    if (e) return set_error(PR_ERR_HIP, "exchange regroup: %s", hipGetErrorString((hipError_t)e));
    std::vector<int32_t> cnt((size_t)c->n_lr + 1, 0);
    int32_t err = 0;
    if (c->n_lr) HIPCHK(hipMemcpyAsync(cnt.data(), R.cnt, (size_t)c->n_lr * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&err, R.err, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (err) return set_error(PR_ERR_ARG, "exchange: a received alignment lies outside the owned long reads");
    int mx = 0;
    for (int i = 0; i < c->n_lr; ++i) mx = std::max(mx, cnt[(size_t)i]);
    std::memset(sp, 0, sizeof *sp);
    sp->t_sr = R.o_sr;
    sp->status = R.o_status;
    sp->pos = R.o_pos;
    sp->score = R.o_score;
    sp->ncig = R.o_ncig;
    sp->cig_at = R.o_cig_at;
    sp->strand = R.o_strand;
    sp->pass = R.o_pass;
    sp->sr_off = B[XB_SROFF].as<int64_t>();
    sp->cig = B[XB_RCIG].as<uint32_t>();
    sp->n_task = R.n;
    sp->task_off = R.task_off;
    sp->max_per_lr = mx;
    return 0;
}

extern "C" int pr_iter_launch(pr_ctx *c, const pr_sw_opts *o, const pr_cns_params *p) {
    if (!c || !o || !p) return set_error(PR_ERR_ARG, "null arg");
    if (!c->pipe) return set_error(PR_ERR_ARG, "no resident iteration batch (pr_iter_upload first)");
    int rc;
    SwPtrs sp;
    if (c->own) {   // owned batch: the SW and the exchange ran before (ev[0]: the exchange's start)
        HIPCHK(hipSetDevice(c->device));
        if ((rc = own_group(c, &sp))) return rc;
    } else {
        if ((rc = pr_sw_launch(c, o))) return rc;   // records ev[2], ev[3], ev[0]
        if ((rc = sw_get_pipe_ptrs(c, &sp, true))) return rc;
    }
    if (sp.task_off) {   // bwa mode: the reported alignments grouped by long read on the device
        if (sp.max_per_lr > 16384)
            return set_error(PR_ERR_CAPACITY, "more than 16384 alignments on one long read (%d)", sp.max_per_lr);
        c->k_need = sp.max_per_lr > 1 ? sp.max_per_lr : 1;
        int sc = 1;
        while (sc < c->k_need) sc <<= 1;
        c->pipe_sort_cap = sc;
    }
    DevBuf *B = c->cb;
    PipeDev P;
    P.n_lr = c->n_lr;
    P.sort_cap = c->pipe_sort_cap;
    P.cig_at = sp.cig_at;
    P.task_off = sp.task_off ? sp.task_off : c->pb[0].as<int64_t>();
    P.t_sr = sp.t_sr;
    P.strand = sp.strand;
    P.pass = sp.pass;
    P.status = sp.status;
    P.pos = sp.pos;
    P.score = sp.score;
    P.ncig = sp.ncig;
    P.sr_off = sp.sr_off;
    P.cnt = c->pb[1].as<int32_t>();
    P.aln_off = B[CB_ALN_OFF].as<int64_t>();
    P.err = c->pb[2].as<int32_t>();
    P.a_pos = B[CB_POS].as<int32_t>();
    P.a_score = B[CB_SCORE].as<double>();
    P.a_flags = B[CB_AFLAGS].as<uint8_t>();
    P.a_seq_off = B[CB_SEQ_OFF].as<int64_t>();
    P.a_lseq = B[CB_LSEQ].as<int32_t>();
    P.a_cig_off = B[CB_CIG_OFF].as<int64_t>();
    P.a_ncig = B[CB_NCIG].as<int32_t>();
    P.lr_off = B[CB_LR_OFF].as<int64_t>();
    P.cig = sp.cig;
    P.keep = nullptr;
    if (c->n_lr == 0) return 0;
    const int grid = c->n_lr < c->n_cu * 4 ? c->n_lr : c->n_cu * 4;
    HIPCHK(hipMemsetAsync(c->pb[2].p, 0, (size_t)c->n_lr * 4, c->stream));
    if (o->bin_size > 0 && o->bin_length > 0) {   // bwa-proovread -b/-l (bin/proovread:1302-1313)
        const size_t nt1 = (size_t)sp.n_task + 1;
        if ((rc = c->pb[3].ensure(nt1)) || (rc = c->pb[4].ensure(nt1 * 4)) || (rc = c->pb[5].ensure(nt1 * 4)) ||
            (rc = c->pb[6].ensure(nt1 * 8)) || (rc = c->pb[7].ensure(nt1 * 4)) || (rc = c->pb[8].ensure(nt1 * 8)) ||
            (rc = c->pb[9].ensure(nt1 * 4)))
            return rc;
        int64_t lmax = 0;
        for (int i = 0; i < c->n_lr; ++i) lmax = std::max(lmax, c->lr_off_host[i + 1] - c->lr_off_host[i]);
        const int64_t max_bins = (lmax + 1024) / o->bin_size + 2;
        if ((2 * max_bins + 256) * 4 > 160 * 1024)
            return set_error(PR_ERR_CAPACITY, "-b/-l filter: %lld bins per long read exceed the LDS layout",
                             (long long)max_bins);
        P.keep = c->pb[3].as<uint8_t>();
        P.fsorted = c->pb[4].as<int32_t>();
        P.fbin = c->pb[5].as<int32_t>();
        P.fnc = c->pb[6].as<double>();
        P.flen = c->pb[7].as<int32_t>();
        P.flst = c->pb[8].as<double>();
        P.flsti = c->pb[9].as<int32_t>();
        // (latency-bound, a few KB of LDS per workgroup: 8 workgroups per CU)
        const int grid_f = c->n_lr < c->n_cu * 8 ? c->n_lr : c->n_cu * 8;
        int e = pipe_binfilter_launch(P, o->bin_size, o->bin_length, (int)max_bins, grid_f, (void *)c->stream);
        if (e) return set_error(PR_ERR_HIP, "-b/-l filter kernel: %s", hipGetErrorString((hipError_t)e));
    }
    c->cns_gathered = false;   // the hand-off writes offsets into the SW / short-read pools
    int e = pipe_launch(P, grid, (void *)c->stream, c->pipe_sort_cap * 8);
    if (e) return set_error(PR_ERR_HIP, "pipe kernels: %s", hipGetErrorString((hipError_t)e));
    return pr_cns_launch(c, p);
}

int sw_keep_to_sam(pr_ctx *c, const uint8_t *keep_grouped, uint8_t *keep_sam);

// bwa-proovread -b/-l on the last bwa-mode SW launch alone (the `mem` drop-in): the hand-off's
// grouping by long read and pipe_binfilter_kernel, as pr_iter_launch runs them
extern "C" int pr_sw_binfilter(pr_ctx *c, int32_t bin_size, double bin_length, uint8_t *keep) {
    if (!c || !keep) return set_error(PR_ERR_ARG, "null arg");
    if (bin_size <= 0 || !(bin_length > 0)) return set_error(PR_ERR_ARG, "-b / -l must be positive");
    HIPCHK(hipSetDevice(c->device));
    SwPtrs sp;
    int rc;
    if ((rc = sw_get_pipe_ptrs(c, &sp, true))) return rc;
    if (!sp.task_off) return set_error(PR_ERR_ARG, "pr_sw_binfilter: bwa mode only");
    const int n_lr = sp.n_lr;
    if (n_lr == 0 || sp.n_task == 0) return 0;
    std::vector<int64_t> lo((size_t)n_lr + 1);
    HIPCHK(hipMemcpyAsync(lo.data(), sp.lr_off, ((size_t)n_lr + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    int64_t lmax = 0;
    for (int i = 0; i < n_lr; ++i) lmax = std::max(lmax, lo[(size_t)i + 1] - lo[(size_t)i]);
    const int64_t max_bins = (lmax + 1024) / bin_size + 2;
    if ((2 * max_bins + 256) * 4 > 160 * 1024)
        return set_error(PR_ERR_CAPACITY, "-b/-l filter: %lld bins per long read exceed the LDS layout", (long long)max_bins);
    const size_t nt1 = (size_t)sp.n_task + 1;
    if ((rc = c->pb[2].ensure(((size_t)n_lr + 1) * 4)) || (rc = c->pb[3].ensure(nt1)) || (rc = c->pb[4].ensure(nt1 * 4)) ||
        (rc = c->pb[5].ensure(nt1 * 4)) || (rc = c->pb[6].ensure(nt1 * 8)) || (rc = c->pb[7].ensure(nt1 * 4)) ||
        (rc = c->pb[8].ensure(nt1 * 8)) || (rc = c->pb[9].ensure(nt1 * 4)))
        return rc;
    PipeDev P;
    std::memset(&P, 0, sizeof P);
    P.n_lr = n_lr;
    P.task_off = sp.task_off;
    P.t_sr = sp.t_sr;
    P.strand = sp.strand;
    P.pass = sp.pass;
    P.status = sp.status;
    P.pos = sp.pos;
    P.score = sp.score;
    P.ncig = sp.ncig;
    P.sr_off = sp.sr_off;
    P.cig_at = sp.cig_at;
    P.lr_off = sp.lr_off;
    P.cig = sp.cig;
    P.err = c->pb[2].as<int32_t>();
    P.keep = c->pb[3].as<uint8_t>();
    P.fsorted = c->pb[4].as<int32_t>();
    P.fbin = c->pb[5].as<int32_t>();
    P.fnc = c->pb[6].as<double>();
    P.flen = c->pb[7].as<int32_t>();
    P.flst = c->pb[8].as<double>();
    P.flsti = c->pb[9].as<int32_t>();
    HIPCHK(hipMemsetAsync(c->pb[2].p, 0, (size_t)n_lr * 4, c->stream));
    const int grid_f = n_lr < c->n_cu * 8 ? n_lr : c->n_cu * 8;
    const int e = pipe_binfilter_launch(P, bin_size, bin_length, (int)max_bins, grid_f, (void *)c->stream);
    if (e) return set_error(PR_ERR_HIP, "-b/-l filter kernel: %s", hipGetErrorString((hipError_t)e));
    std::vector<int32_t> err((size_t)n_lr);
    HIPCHK(hipMemcpyAsync(err.data(), c->pb[2].p, (size_t)n_lr * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < n_lr; ++i)
        if (err[(size_t)i]) return set_error(PR_ERR_CAPACITY, "-b/-l filter of long read %d failed (code %d)", i, err[(size_t)i]);
    return sw_keep_to_sam(c, c->pb[3].as<uint8_t>(), keep);
}

extern "C" int pr_iter_download(pr_ctx *c, pr_cns_out *o) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    int rc = pr_cns_download(c, o);
    if (rc || !c->pipe || !c->n_lr) return rc;
    // the hand-off's per-read error flags (sort capacity, filter bin range): never silent
    std::vector<int32_t> err((size_t)c->n_lr);
    HIPCHK(hipMemcpy(err.data(), c->pb[2].p, (size_t)c->n_lr * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < c->n_lr; ++i)
        if (err[(size_t)i]) return set_error(PR_ERR_CAPACITY, "hand-off of long read %d failed (code %d)", i, err[(size_t)i]);
    return 0;
}

extern "C" int pr_iter_download_range(pr_ctx *c, int32_t first, int32_t n, pr_cns_out *o) {
    // reads [first, first + n) of the last launch: the per-read arrays have n entries, out_off /
    // chim_off n + 1 entries counted from the range's first read
    if (!c || !o) return set_error(PR_ERR_ARG, "null arg");
    if (first < 0 || n < 0 || (int64_t)first + n > c->n_lr) return set_error(PR_ERR_ARG, "read range outside the batch");
    if (o->kept || o->bin_bases) return set_error(PR_ERR_ARG, "kept / bin_bases: pr_iter_download");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
    if (!c->cns_launched) return set_error(PR_ERR_ARG, "no consensus launch to download");
    const size_t f = (size_t)first, m = (size_t)n;
    const int64_t o0 = c->out_off[f], o1 = c->out_off[f + m], h0 = c->chim_off[f], h1 = c->chim_off[f + m];
    if (o->out_off)
        for (size_t i = 0; i <= m; ++i) o->out_off[i] = c->out_off[f + i] - o0;
    if (o->chim_off)
        for (size_t i = 0; i <= m; ++i) o->chim_off[i] = c->chim_off[f + i] - h0;
    DevBuf *B = c->cb;
    int rc;
    if ((rc = download(o->status, B[CB_STATUS], m, s, f)) || (rc = download(o->seq_len, B[CB_SEQ_LEN], m, s, f)) ||
        (rc = download(o->trace_len, B[CB_TRACE_LEN], m, s, f)) || (rc = download(o->ncigar, B[CB_NCIGAR], m, s, f)) ||
        (rc = download(o->nchim, B[CB_NCHIM], m, s, f)) || (rc = download(o->seq, B[CB_O_SEQ], (size_t)(o1 - o0), s, (size_t)o0)) ||
        (rc = download(o->qual, B[CB_O_QUAL], (size_t)(o1 - o0), s, (size_t)o0)) ||
        (rc = download(o->trace, B[CB_O_TRACE], (size_t)(o1 - o0), s, (size_t)o0)) ||
        (rc = download(o->cigar, B[CB_O_CIG], (size_t)(o1 - o0), s, (size_t)o0)) ||
        (rc = download(o->chim, B[CB_O_CHIM], (size_t)(h1 - h0) * 4, s, (size_t)h0 * 4)))
        return rc;
    std::vector<int32_t> err(m + 1, 0);
    if (c->pipe && m) HIPCHK(hipMemcpyAsync(err.data(), c->pb[2].as<int32_t>() + f, m * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (size_t i = 0; i < m; ++i)
        if (err[i]) return set_error(PR_ERR_CAPACITY, "hand-off of long read %d failed (code %d)", first + (int)i, err[i]);
    return 0;
}

extern "C" int pr_iter_last_timing(pr_ctx *c, double *ms_sw_extend, double *ms_sw_global, double *ms_assemble,
                                   double *ms_consensus) {
    // HIP events of the last pr_iter_launch (the caller has synchronised):
    // ev2 | SW extend | ev3 | SW global | ev0 | hand-off | ev4 | consensus | ev5
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    const int pairs[4][2] = {{2, 3}, {3, 0}, {0, 4}, {4, 5}};
    for (int k = 0; k < 4; ++k)
        if (hipEventElapsedTime(&v[k], c->ev[pairs[k][0]], c->ev[pairs[k][1]]) != hipSuccess) v[k] = 0.f;
    if (ms_sw_extend) *ms_sw_extend = v[0];
    if (ms_sw_global) *ms_sw_global = v[1];
    if (ms_assemble) *ms_assemble = v[2];
    if (ms_consensus) *ms_consensus = v[3];
    return 0;
}

extern "C" int pr_iter_alignment_stats(pr_ctx *c, int64_t *n_aln, int64_t *sum_ncig, int64_t *sum_lseq) {
    // reported alignments of the last iteration (for the SURVEY.md §8d pileup byte model)
    if (!c || !c->pipe) return set_error(PR_ERR_ARG, "no resident iteration batch");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    int64_t na = 0;
    HIPCHK(hipMemcpy(&na, c->cb[CB_ALN_OFF].as<int64_t>() + c->n_lr, 8, hipMemcpyDeviceToHost));
    std::vector<int32_t> v((size_t)na + 1);
    int64_t sc = 0, sl = 0;
    if (na) {
        HIPCHK(hipMemcpy(v.data(), c->cb[CB_NCIG].p, (size_t)na * 4, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < na; ++i) sc += v[i];
        HIPCHK(hipMemcpy(v.data(), c->cb[CB_LSEQ].p, (size_t)na * 4, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < na; ++i) sl += v[i];
    }
    if (n_aln) *n_aln = na;
    if (sum_ncig) *sum_ncig = sc;
    if (sum_lseq) *sum_lseq = sl;
    return 0;
}

extern "C" int pr_iter_bounds(pr_ctx *c, int32_t *n_lr, int64_t *n_task, pr_cns_bounds *bd) {
    if (!c || !c->pipe) return set_error(PR_ERR_ARG, "no resident iteration batch");
    if (n_lr) *n_lr = c->n_lr;
    if (n_task) *n_task = c->n_aln;
    if (bd) { bd->seq_cap = c->seq_cap; bd->chim_cap = c->chim_cap; }
    return 0;
}

extern "C" int pr_ctx_sync(pr_ctx *c) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipGetLastError());
    return 0;
}

extern "C" int pr_dev_alloc(pr_ctx *c, int64_t bytes, void **dev) {
    if (!c || !dev || bytes < 0) return set_error(PR_ERR_ARG, "bad arg");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMalloc(dev, (size_t)(bytes ? bytes : 16)));
    HIPCHK(hipMemsetAsync(*dev, 0, (size_t)(bytes ? bytes : 16), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int pr_dev_free(pr_ctx *c, void *dev) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (dev) HIPCHK(hipFree(dev));
    return 0;
}

extern "C" int pr_dev_download(pr_ctx *c, void *host, const void *dev, int64_t bytes) {
    if (!c || bytes < 0 || (bytes && (!host || !dev))) return set_error(PR_ERR_ARG, "bad arg");
    HIPCHK(hipSetDevice(c->device));
    if (bytes) HIPCHK(hipMemcpyAsync(host, dev, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int pr_dev_upload(pr_ctx *c, void *dev, const void *host, int64_t bytes) {
    if (!c || bytes < 0 || (bytes && (!host || !dev))) return set_error(PR_ERR_ARG, "bad arg");
    HIPCHK(hipSetDevice(c->device));
    if (bytes) HIPCHK(hipMemcpyAsync(dev, host, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" int pr_iter_stats(pr_ctx *c, int32_t min_phred, int64_t *dev_out) {
    if (!c || !dev_out) return set_error(PR_ERR_ARG, "null arg");
    if (!c->cns_loaded) return set_error(PR_ERR_ARG, "no resident consensus batch");
    HIPCHK(hipSetDevice(c->device));
    DevBuf *B = c->cb;
    int e = iter_stats_launch(B[CB_OUT_OFF].as<int64_t>(), B[CB_STATUS].as<int32_t>(), B[CB_SEQ_LEN].as<int32_t>(),
                              B[CB_O_QUAL].as<uint8_t>(), c->n_lr, min_phred + 33,
                              reinterpret_cast<unsigned long long *>(dev_out), (void *)c->stream);
    if (e) return set_error(PR_ERR_HIP, "stats kernel: %s", hipGetErrorString((hipError_t)e));
    return 0;
}

// ---------------------------------------------------------------------------
// masking (SeqFilter --phred-mask of bin/proovread:1701-1716; mask_core.h)
extern "C" void pr_mask_params_default(pr_mask_params *p) {
    p->phred_min = 20;        // proovread.cfg:235 "20,41,80,130,60,0.7" at 100 bp short reads
    p->phred_max = 41;
    p->mask_min_len = 80;
    p->unmask_min_len = 130;
    p->mask_reduce = 60;
    p->end_ratio = 0.7;
    p->phred_offset = 33;
}

extern "C" int pr_mask_params_parse(const char *hcr_mask, int32_t min_sr_length, pr_mask_params *out) {
    if (!hcr_mask || !out || min_sr_length <= 0) return set_error(PR_ERR_ARG, "hcr_mask, out and min_sr_length > 0");
    double f[6];
    const char *q = hcr_mask;
    for (int i = 0; i < 6; ++i) {
        char *e = nullptr;
        f[i] = std::strtod(q, &e);
        if (e == q || (i < 5 && *e != ',') || (i == 5 && *e && *e != '\n'))
            return set_error(PR_ERR_ARG, "hcr-mask '%s': want phred-min,phred-max,mask-min-len,unmask-min-len,"
                             "mask-reduce,mask-end-ratio", hcr_mask);
        q = e + 1;
    }
    pr_mask_params_default(out);
    out->phred_min = (int32_t)f[0];
    out->phred_max = (int32_t)f[1];
    // proovread:1703-1704: int(x * min_sr_length / 100 + .5)
    out->mask_min_len = (int32_t)(f[2] * min_sr_length / 100.0 + .5);
    out->unmask_min_len = (int32_t)(f[3] * min_sr_length / 100.0 + .5);
    out->mask_reduce = (int32_t)f[4];
    out->end_ratio = f[5];
    return 0;
}

static int mask_cfg(const pr_mask_params *p, MaskCfg *c) {
    if (!p) return set_error(PR_ERR_ARG, "null params");
    if (p->mask_min_len < 1 || p->mask_reduce < 0 || p->unmask_min_len < 0 || p->phred_min > p->phred_max)
        return set_error(PR_ERR_ARG, "mask params: need mask_min_len >= 1, mask_reduce >= 0, unmask_min_len >= 0, "
                         "phred_min <= phred_max");
    c->lo_char = p->phred_min + p->phred_offset;
    c->hi_char = p->phred_max + p->phred_offset;
    c->lcs_min = p->mask_min_len + 2 * p->mask_reduce;
    c->hcr_min = p->mask_min_len;
    c->lcr_min = p->unmask_min_len;
    c->sticky = p->mask_reduce;
    c->end_ratio = p->end_ratio;
    return 0;
}

static void mask_run_offsets(const int64_t *off, int32_t n, int32_t lcs_min, std::vector<int64_t> &ro) {
    ro.assign((size_t)n + 1, 0);
    for (int32_t i = 0; i < n; ++i) ro[i + 1] = ro[i] + mask_run_cap(off[i + 1] - off[i], lcs_min);
}

extern "C" int pr_mask_bound(const pr_mask_params *p, int32_t n, const int64_t *off, int64_t *mcr_cap) {
    MaskCfg mc;
    int rc = mask_cfg(p, &mc);
    if (rc) return rc;
    if (n < 0 || (n && !off) || !mcr_cap) return set_error(PR_ERR_ARG, "bad batch");
    std::vector<int64_t> ro;
    mask_run_offsets(off, n, mc.lcs_min, ro);
    *mcr_cap = ro[n];
    return 0;
}

static int mask_enqueue(pr_ctx *c, MaskDev &D, const std::vector<int64_t> &ro) {
    DevBuf *M = c->mb;
    hipStream_t s = c->stream;
    const int64_t nr = ro.back();
    int rc;
    if ((rc = upload(M[MB_RUN_OFF], ro.data(), ro.size(), s)) || (rc = M[MB_RUNS].ensure((size_t)nr * 8)) ||
        (rc = M[MB_TMP].ensure((size_t)nr * 8)) || (rc = M[MB_NRUNS].ensure((size_t)(D.n > 0 ? D.n : 1) * 4)) ||
        (rc = M[MB_ERR].ensure(4)) || (rc = M[MB_STATS].ensure(16)))
        return rc;
    D.run_off = M[MB_RUN_OFF].as<int64_t>();
    D.runs = M[MB_RUNS].as<MaskRun>();
    D.tmp = M[MB_TMP].as<MaskRun>();
    D.n_runs = M[MB_NRUNS].as<int32_t>();
    D.err = M[MB_ERR].as<int32_t>();
    if (!D.stats) D.stats = M[MB_STATS].as<unsigned long long>();
    const int e = mask_launch(D, c->n_cu, (void *)s);
    if (e) return set_error(PR_ERR_HIP, "mask kernel: %s", hipGetErrorString((hipError_t)e));
    return 0;
}

static int mask_check_err(pr_ctx *c) {
    int32_t err = 0;
    HIPCHK(hipMemcpyAsync(&err, c->mb[MB_ERR].p, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (err) return set_error(PR_ERR_CAPACITY, "masking: HCR list exceeded its run capacity");
    return 0;
}

extern "C" int pr_mask_run(pr_ctx *c, const pr_mask_params *p, int32_t n, const int64_t *off, const uint8_t *seq,
                           const uint8_t *qual, uint8_t *out_seq, int64_t *mcr_off, int32_t *mcr, int32_t *n_mcr,
                           int64_t *stats) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    MaskCfg mc;
    int rc = mask_cfg(p, &mc);
    if (rc) return rc;
    if (n < 0 || (n && (!off || !seq || !qual))) return set_error(PR_ERR_ARG, "bad batch");
    if (n && off[0] != 0) return set_error(PR_ERR_ARG, "offsets must start at 0");
    for (int32_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) return set_error(PR_ERR_ARG, "offsets not monotone at %d", i);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const int64_t nb = n ? off[n] : 0;
    DevBuf *M = c->mb;
    if ((rc = upload(M[MB_OFF], off, (size_t)n + 1, s)) || (rc = upload(M[MB_SEQ], seq, (size_t)nb, s)) ||
        (rc = upload(M[MB_QUAL], qual, (size_t)nb, s)) || (rc = M[MB_OUT].ensure((size_t)nb)))
        return rc;
    std::vector<int64_t> ro;
    mask_run_offsets(n ? off : nullptr, n, mc.lcs_min, ro);
    MaskDev D{};
    D.n = n;
    D.off = M[MB_OFF].as<int64_t>();
    D.seq = M[MB_SEQ].as<uint8_t>();
    D.qual = M[MB_QUAL].as<uint8_t>();
    D.out = M[MB_OUT].as<uint8_t>();
    D.cfg = mc;
    if ((rc = mask_enqueue(c, D, ro))) return rc;
    if ((rc = mask_check_err(c))) return rc;
    unsigned long long st[2] = {0, 0};
    if ((rc = download(out_seq, M[MB_OUT], (size_t)nb, s)) || (rc = download(n_mcr, M[MB_NRUNS], (size_t)n, s)) ||
        (rc = download(reinterpret_cast<MaskRun *>(mcr), M[MB_RUNS], (size_t)ro[n], s)))
        return rc;
    HIPCHK(hipMemcpyAsync(st, M[MB_STATS].p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (mcr_off) std::memcpy(mcr_off, ro.data(), ro.size() * sizeof(int64_t));
    if (stats) {
        stats[0] = (int64_t)st[0];
        stats[1] = (int64_t)st[1];
    }
    return 0;
}

extern "C" int pr_iter_mask(pr_ctx *c, const pr_mask_params *p, int64_t *dev_stats) {
    if (!c) return set_error(PR_ERR_ARG, "null ctx");
    if (!c->cns_loaded || !c->cns_launched) return set_error(PR_ERR_ARG, "no consensus launch to mask");
    MaskCfg mc;
    int rc = mask_cfg(p, &mc);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    DevBuf *B = c->cb;
    if ((rc = c->mb[MB_OUT].ensure((size_t)(c->seq_cap > 0 ? c->seq_cap : 1)))) return rc;
    std::vector<int64_t> ro;
    mask_run_offsets(c->out_off.data(), c->n_lr, mc.lcs_min, ro);
    MaskDev D{};
    D.n = c->n_lr;
    D.off = B[CB_OUT_OFF].as<int64_t>();
    D.len = B[CB_SEQ_LEN].as<int32_t>();
    D.status = B[CB_STATUS].as<int32_t>();
    D.seq = B[CB_O_SEQ].as<uint8_t>();
    D.qual = B[CB_O_QUAL].as<uint8_t>();
    D.out = c->mb[MB_OUT].as<uint8_t>();
    D.stats = reinterpret_cast<unsigned long long *>(dev_stats);
    D.cfg = mc;
    if ((rc = mask_enqueue(c, D, ro))) return rc;
    c->iter_masked = true;
    return 0;
}

extern "C" int pr_iter_mask_download(pr_ctx *c, uint8_t *masked) {
    if (!c || !masked) return set_error(PR_ERR_ARG, "null arg");
    if (!c->iter_masked) return set_error(PR_ERR_ARG, "no pr_iter_mask launch yet");
    HIPCHK(hipSetDevice(c->device));
    int rc = mask_check_err(c);
    if (rc) return rc;
    if ((rc = download(masked, c->mb[MB_OUT], (size_t)c->seq_cap, c->stream))) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

static int index_build(pr_ctx *c, const uint8_t *lr_seq, const int64_t *lr_off, int n_lr, bool lr_dev);

// ---------------------------------------------------------------------------
// the resident long-read set (include/prgpu.h pr_lrset_*): the loop's LR.fq and LR.masked.fa
// between tasks, in HBM
extern "C" int pr_lrset_load(pr_ctx *c, int32_t n_lr, const int64_t *off, const uint8_t *seq, const uint8_t *qual) {
    if (!c || n_lr < 0 || !off || (n_lr && (!seq || !qual))) return set_error(PR_ERR_ARG, "null arg");
    if (off[0] != 0) return set_error(PR_ERR_ARG, "offsets must start at 0");
    for (int i = 0; i < n_lr; ++i)
        if (off[i + 1] < off[i]) return set_error(PR_ERR_ARG, "offsets not monotone");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t nb = (size_t)off[n_lr];
    int rc;
    if ((rc = upload(c->ls[LS_SEQ], seq, nb, s)) || (rc = upload(c->ls[LS_QUAL], qual, nb, s))) return rc;
    HIPCHK(hipStreamSynchronize(s));
    c->ls_off.assign(off, off + n_lr + 1);
    c->ls_n = n_lr;
    c->ls_map_is_reads = true;   // read-long: the mapping reference is the reads themselves
    return 0;
}

extern "C" int pr_lrset_snapshot(pr_ctx *c) {
    if (!c || c->ls_n < 0) return set_error(PR_ERR_ARG, "no resident long-read set (pr_lrset_load)");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t nb = (size_t)c->ls_off.back();
    int rc;
    if ((rc = c->ls[LS_RSEQ].ensure(nb + 1)) || (rc = c->ls[LS_RQUAL].ensure(nb + 1))) return rc;
    if (nb) {
        HIPCHK(hipMemcpyAsync(c->ls[LS_RSEQ].p, c->ls[LS_SEQ].p, nb, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(c->ls[LS_RQUAL].p, c->ls[LS_QUAL].p, nb, hipMemcpyDeviceToDevice, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    c->ls_raw_off = c->ls_off;
    return 0;
}

extern "C" int pr_lrset_restore(pr_ctx *c) {
    if (!c || c->ls_n < 0) return set_error(PR_ERR_ARG, "no resident long-read set (pr_lrset_load)");
    if (c->ls_raw_off.empty()) return set_error(PR_ERR_ARG, "no snapshot of the long-read set (pr_lrset_snapshot)");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t nb = (size_t)c->ls_raw_off.back();
    int rc;
    if ((rc = c->ls[LS_SEQ].ensure(nb + 1)) || (rc = c->ls[LS_QUAL].ensure(nb + 1))) return rc;
    if (nb) {   // stream-ordered after every launch that read the set
        HIPCHK(hipMemcpyAsync(c->ls[LS_SEQ].p, c->ls[LS_RSEQ].p, nb, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(c->ls[LS_QUAL].p, c->ls[LS_RQUAL].p, nb, hipMemcpyDeviceToDevice, s));
    }
    c->ls_off = c->ls_raw_off;
    c->ls_n = (int32_t)c->ls_off.size() - 1;
    c->ls_map_is_reads = true;   // read-long: the mapping reference is the reads themselves
    return 0;
}

extern "C" int pr_lrset_info(pr_ctx *c, int32_t *n_lr, int64_t *bases) {
    if (!c || c->ls_n < 0) return set_error(PR_ERR_ARG, "no resident long-read set (pr_lrset_load)");
    if (n_lr) *n_lr = c->ls_n;
    if (bases) *bases = c->ls_off.back();
    return 0;
}

extern "C" int pr_lrset_download(pr_ctx *c, int64_t *off, uint8_t *seq, uint8_t *qual, uint8_t *map) {
    if (!c || c->ls_n < 0) return set_error(PR_ERR_ARG, "no resident long-read set (pr_lrset_load)");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t nb = (size_t)c->ls_off.back();
    if (off) std::memcpy(off, c->ls_off.data(), c->ls_off.size() * 8);
    int rc;
    if ((rc = download(seq, c->ls[LS_SEQ], nb, s)) || (rc = download(qual, c->ls[LS_QUAL], nb, s)) ||
        (rc = download(map, c->ls[c->ls_map_is_reads ? LS_SEQ : LS_MAP], nb, s)))
        return rc;
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

extern "C" int pr_lrset_index(pr_ctx *c, int which) {
    if (!c || c->ls_n < 0) return set_error(PR_ERR_ARG, "no resident long-read set (pr_lrset_load)");
    if (which != PR_LRSET_MAP && which != PR_LRSET_READS) return set_error(PR_ERR_ARG, "which: PR_LRSET_MAP / _READS");
    const int id = which == PR_LRSET_READS || c->ls_map_is_reads ? LS_SEQ : LS_MAP;
    return index_build(c, c->ls[id].as<uint8_t>(), c->ls_off.data(), c->ls_n, true);
}

extern "C" int pr_iter_upload_lrset(pr_ctx *c, const pr_sw_batch *b) {
    if (!c || !b) return set_error(PR_ERR_ARG, "null arg");
    if (c->ls_n < 0) return set_error(PR_ERR_ARG, "no resident long-read set (pr_lrset_load)");
    if (!c->seed_n_text || c->seed_view.n_lr != c->ls_n || c->seed_view.l_pac != c->ls_off.back())
        return set_error(PR_ERR_ARG, "the seed index is not over the long-read set (pr_lrset_index first)");
    if (c->seed_pre.size() != (size_t)b->n_sr + 1)
        return set_error(PR_ERR_ARG, "no device seeds for these short reads (pr_seed_gpu_map with out = NULL first)");
    if (!b->sr_seq && b->n_sr && c->seed_sr_bases != b->sr_off[b->n_sr])
        return set_error(PR_ERR_ARG, "sr_seq NULL: the short reads must be those of the last pr_seed_gpu_map");
    pr_iter_batch ib;
    std::memset(&ib, 0, sizeof ib);
    ib.sw = *b;
    ib.sw.n_lr = c->ls_n;
    ib.sw.lr_off = c->ls_off.data();
    ib.sw.lr_seq = nullptr;
    const int rc = iter_upload(c, &ib, true, b->sr_seq ? nullptr : c->sd[SB_SEQ].as<uint8_t>(),
                               c->sd[SX_LRSEQ].as<uint8_t>(), c->ls[LS_SEQ].as<uint8_t>(), c->ls[LS_QUAL].as<uint8_t>());
    if (!rc && !b->sr_seq) c->seed_sr_bases = -1;   // handed over once (as pr_sw_upload_gpu_seeds)
    return rc;
}

// pr_lrset_commit's checks on this rank: the launch, the masking, every read's hand-off and
// consensus status (as pr_iter_download: never silent); fills the per-read status and length
static int commit_check(pr_ctx *c, int world, bool with_mask, int lr0, int n, std::vector<int32_t> &st,
                        std::vector<int32_t> &len, std::vector<int32_t> &herr) {
    if (!c->cns_launched || !c->pipe) return set_error(PR_ERR_ARG, "no iteration launch to commit");
    if (with_mask && !c->iter_masked) return set_error(PR_ERR_ARG, "with_mask: no pr_iter_mask launch");
    if (world == 1 && (lr0 != 0 || n != c->ls_n)) return set_error(PR_ERR_ARG, "the batch must hold every long read");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if (with_mask && (rc = mask_check_err(c))) return rc;
    if (n) {
        HIPCHK(hipMemcpyAsync(st.data(), c->cb[CB_STATUS].p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(len.data(), c->cb[CB_SEQ_LEN].p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(herr.data(), c->pb[2].p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i) {
        if (herr[(size_t)i])
            return set_error(PR_ERR_CAPACITY, "hand-off of long read %d failed (code %d)", lr0 + i, herr[(size_t)i]);
        if (st[(size_t)i]) return set_error(st[(size_t)i], "consensus of long read %d failed (status %d)", lr0 + i, st[(size_t)i]);
    }
    return 0;
}

extern "C" int pr_lrset_commit(pr_ctx *c, pr_comm *comm, int flags) {
    if (!c || c->ls_n < 0) return set_error(PR_ERR_ARG, "no resident long-read set (pr_lrset_load)");
    int rank = 0, world = 1, rc;
    if (comm && (rc = pr_comm_rank(comm, &rank, &world))) return rc;
    if (comm && comm_ctx(comm) != c) return set_error(PR_ERR_ARG, "the communicator belongs to another context");
    const bool dry = (flags & PR_LRSET_COMMIT_DRY) != 0, with_mask = (flags & PR_LRSET_COMMIT_MASK) != 0;
    const int lr0 = c->own ? c->own_lr0 : 0, n = c->n_lr;
    std::vector<int32_t> st((size_t)n + 1, 0), len((size_t)n + 1, 0), herr((size_t)n + 1, 0);
    // local checks first; with ranks, every rank learns whether all passed before any collective
    rc = commit_check(c, world, with_mask, lr0, n, st, len, herr);
    if (world > 1) rc = pr_comm_agree(comm, rc);
    if (rc) return rc;
    hipStream_t s = c->stream;
    std::vector<int64_t> doff((size_t)n + 1, 0);
    for (int i = 0; i < n; ++i) doff[(size_t)i + 1] = doff[(size_t)i] + len[(size_t)i];
    const int64_t own = doff[(size_t)n];
    DevBuf *L = c->ls;
    // the compaction's buffers and launch are local too: with ranks, agree again before the
    // first collective so a rank that failed here does not leave the others inside it
    if (!(rc = upload(L[LS_OFF], doff.data(), (size_t)n + 1, s)) && !(rc = L[LS_TSEQ].ensure((size_t)own + 1)) &&
        !(rc = L[LS_TQUAL].ensure((size_t)own + 1)) && !(with_mask && (rc = L[LS_TMAP].ensure((size_t)own + 1)))) {
        const int e = lr_compact_launch(c->cb[CB_OUT_OFF].as<int64_t>(), c->cb[CB_SEQ_LEN].as<int32_t>(),
                                        L[LS_OFF].as<int64_t>(), n, c->cb[CB_O_SEQ].as<uint8_t>(), L[LS_TSEQ].as<uint8_t>(),
                                        c->cb[CB_O_QUAL].as<uint8_t>(), L[LS_TQUAL].as<uint8_t>(),
                                        with_mask ? c->mb[MB_OUT].as<uint8_t>() : nullptr,
                                        with_mask ? L[LS_TMAP].as<uint8_t>() : nullptr, (void *)s);
        if (e) rc = set_error(PR_ERR_HIP, "long-read set compaction: %s", hipGetErrorString((hipError_t)e));
    }
    if (world > 1) rc = pr_comm_agree(comm, rc);
    if (rc) return rc;
    std::vector<int64_t> off((size_t)c->ls_n + 1, 0);
    if (world == 1) {
        if (!dry) {
            std::swap(L[LS_SEQ], L[LS_TSEQ]);
            std::swap(L[LS_QUAL], L[LS_TQUAL]);
            if (with_mask) std::swap(L[LS_MAP], L[LS_TMAP]);
        }
        off = doff;
    } else {
        // every rank's owned reads in rank order (= global order: the owners' ranges ascend):
        // the lengths all-gathered on the host (small), the pools on the device
        std::vector<int64_t> cnt((size_t)world, 0);
        cnt[(size_t)rank] = n;
        if ((rc = pr_comm_allreduce_host(comm, cnt.data(), world, PR_DT_I64, PR_RED_SUM))) return rc;
        int64_t tot_n = 0;
        for (int r = 0; r < world; ++r) tot_n += cnt[(size_t)r];
        if (tot_n != c->ls_n) return set_error(PR_ERR_ARG, "the ranks' owned reads do not make up the set");
        std::vector<int64_t> lens((size_t)c->ls_n, 0), bytes((size_t)world, 0);
        int64_t first = 0;
        for (int r = 0; r < rank; ++r) first += cnt[(size_t)r];
        for (int i = 0; i < n; ++i) lens[(size_t)(first + i)] = len[(size_t)i];
        if ((rc = pr_comm_allreduce_host(comm, lens.data(), c->ls_n, PR_DT_I64, PR_RED_SUM))) return rc;
        for (int i = 0; i < c->ls_n; ++i) off[(size_t)i + 1] = off[(size_t)i] + lens[(size_t)i];
        int64_t k = 0;
        for (int r = 0; r < world; ++r) {
            bytes[(size_t)r] = off[(size_t)(k + cnt[(size_t)r])] - off[(size_t)k];
            k += cnt[(size_t)r];
        }
        const size_t tot = (size_t)off.back();
        // dry: the same all-gathers into scratch pools, the set unchanged
        const int ids[3][2] = {{LS_TSEQ, dry ? LS_GSEQ : LS_SEQ}, {LS_TQUAL, dry ? LS_GQUAL : LS_QUAL},
                               {LS_TMAP, dry ? LS_GMAP : LS_MAP}};
        const int nq = with_mask ? 3 : 2;
        // every gather target first, then one more agreement: no rank enters an all-gather that
        // another cannot reach for want of memory
        for (int q = 0; q < nq && !rc; ++q) rc = L[ids[q][1]].ensure(tot + 1);
        rc = pr_comm_agree(comm, rc);
        for (int q = 0; q < nq && !rc; ++q)
            rc = pr_comm_allgatherv_dev(comm, L[ids[q][0]].p, bytes.data(), L[ids[q][1]].p);
        if (dry) {   // the scratch pools of a dry commit are not kept (configs[3]: ~3 x 2.9 GB)
            HIPCHK(hipStreamSynchronize(s));
            for (int q = 0; q < nq; ++q) L[ids[q][1]].release();
        }
        if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(s));
    if (dry) return 0;
    c->ls_off = off;
    if (with_mask) c->ls_map_is_reads = false;
    else c->ls_map_is_reads = true;   // the finish task: the reads are their own mapping reference
    return 0;
}

// ---------------------------------------------------------------------------
// seeding on the device (seed_kernels.hip over seed_core.h)
// the index text 16 bases per word (IndexView.text4) for the occurrence table's match lengths
static int seed_text4(pr_ctx *c, seedc::IndexView &v, hipStream_t s) {
    int rc = c->sd[SI_TEXT4].ensure((size_t)ix_pack4_words(v.n_text) * 8);
    if (rc) return rc;
    const int e = ix_pack4_launch(v.text, v.n_text, c->sd[SI_TEXT4].as<uint64_t>(), s);
    if (e) return set_error(PR_ERR_HIP, "text packing: %s", hipGetErrorString((hipError_t)e));
    v.text4 = c->sd[SI_TEXT4].as<uint64_t>();
    // dense indexes (> 64 hits per 12-mer on average: configs[2] / [3] at one rank's share): the
    // by-wave pass walks 16 bases per text round trip (seed_wave_kernel<1>: no 5-word buffers,
    // more waves resident), the others 64 (tools/ab_scale.sh: profiles/r06_walk_ab.txt)
    v.walk_nw = v.n_text > ((int64_t)64 << 24) ? 1 : 4;
    if (const char *w = getenv("PRGPU_SEED_WALK_NW"))   // tuning hook: 1 or 4
        v.walk_nw = atoi(w) == 1 ? 1 : 4;
    return 0;
}

// Per 2^CB_SHIFT text block: the contig at its start, the next two contig starts inside it and
// the coordinate offsets of those contigs (fr = p + delta, seed_core.h text_to_fr), so the
// seeding's hit pass computes a hit's bwa coordinate with one table load instead of the cblk ->
// cstart -> lr_off chain.  cstart / off: host arrays of the index (off rebased to 0).
static int upload_blk_fr(pr_ctx *c, seedc::IndexView &v, const int64_t *cstart, const int64_t *off, int n_lr,
                         int64_t l_pac, int64_t n_text, hipStream_t s) {
    const int64_t nb = (n_text >> seedc::CB_SHIFT) + 1;
    const int nc = 2 * n_lr;
    const int bs = 1 << seedc::CB_SHIFT;
    auto delta = [&](int ci) -> int64_t {
        if (ci < n_lr) return off[ci] - cstart[ci];
        const int rid = 2 * n_lr - 1 - ci;   // the reverse half holds the long reads in reverse order
        return 2 * l_pac - off[rid + 1] - cstart[ci];
    };
    std::vector<seedc::BlkFr> t((size_t)nb);
    int ci = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t b0 = b << seedc::CB_SHIFT, b1 = b0 + bs;
        while (ci + 1 < nc && cstart[ci + 1] <= b0) ++ci;
        seedc::BlkFr &e = t[(size_t)b];
        e.c0 = ci;
        e.d0 = nc ? delta(ci) : 0;
        e.d1 = ci + 1 < nc ? delta(ci + 1) : 0;
        e.bnd = ci + 1 < nc && cstart[ci + 1] < b1 ? (int32_t)(cstart[ci + 1] - b0) : bs;
        e.bnd2 = ci + 2 < nc && cstart[ci + 2] < b1 ? (int32_t)(cstart[ci + 2] - b0) : bs;
    }
    int rc = c->sd[SI_BLKFR].ensure(t.size() * sizeof(seedc::BlkFr));
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(c->sd[SI_BLKFR].p, t.data(), t.size() * sizeof(seedc::BlkFr), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));   // (t is a host temporary)
    v.blkfr = c->sd[SI_BLKFR].as<seedc::BlkFr>();
    return 0;
}

extern "C" int pr_seed_gpu_upload(pr_ctx *c, const pr_seed_index *h) {
    if (!c || !h) return set_error(PR_ERR_ARG, "null arg");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const seedc::IndexView hv = seed_index_view(h);
    const SeedIndexSizes z = seed_index_sizes(h);
    DevBuf *D = c->sd;
    int rc;
    if ((rc = upload(D[SI_TEXT], hv.text, (size_t)z.text, s)) || (rc = upload(D[SI_CSTART], hv.cstart, (size_t)z.cstart, s)) ||
        (rc = upload(D[SI_CBLK], hv.cblk, (size_t)z.cblk, s)) || (rc = upload(D[SI_LROFF], hv.lr_off, (size_t)z.lr_off, s)) ||
        (rc = upload(D[SI_KOFF], hv.koff, (size_t)z.koff, s)) || (rc = upload(D[SI_KPOS], hv.kpos, (size_t)z.kpos, s)) ||
        (rc = upload(D[SI_KEXT], hv.kext, (size_t)z.kpos, s)) ||
        (z.ksplit && (rc = upload(D[SI_KSPLIT], hv.ksplit, (size_t)z.ksplit, s))))
        return rc;
    seedc::IndexView v = hv;
    for (int j = 0; j < seedc::KI - 1; ++j) {
        if ((rc = upload(D[SI_CNT0 + j], hv.cnt[j], (size_t)z.cnt[j], s))) return rc;
        v.cnt[j] = D[SI_CNT0 + j].as<uint32_t>();
    }
    v.text = D[SI_TEXT].as<uint8_t>();
    v.cstart = D[SI_CSTART].as<int64_t>();
    v.cblk = D[SI_CBLK].as<int32_t>();
    v.lr_off = D[SI_LROFF].as<int64_t>();
    v.koff = D[SI_KOFF].as<uint64_t>();
    v.kpos = D[SI_KPOS].as<uint32_t>();
    v.kext = D[SI_KEXT].as<uint64_t>();
    v.ksplit = z.ksplit ? D[SI_KSPLIT].as<uint64_t>() : nullptr;
    if ((rc = seed_text4(c, v, s))) return rc;
    if ((rc = upload_blk_fr(c, v, hv.cstart, hv.lr_off, hv.n_lr, hv.l_pac, hv.n_text, s))) return rc;
    HIPCHK(hipStreamSynchronize(s));
    c->seed_view = v;
    c->seed_loaded = true;
    return 0;
}

// the seed index built in HBM (seed_index.hip): the tables of pr_seed_index_build
// lr_dev: lr_seq is a device pointer (the resident long-read set), copied on the device
extern "C" int pr_seed_gpu_index_build(pr_ctx *c, const uint8_t *lr_seq, const int64_t *lr_off, int n_lr) {
    return index_build(c, lr_seq, lr_off, n_lr, false);
}

static int index_build(pr_ctx *c, const uint8_t *lr_seq, const int64_t *lr_off, int n_lr, bool lr_dev) {
    if (!c || n_lr < 0 || (n_lr && (!lr_seq || !lr_off))) return set_error(PR_ERR_ARG, "null arg");
    for (int i = 0; i < n_lr; ++i)
        if (lr_off[i + 1] < lr_off[i]) return set_error(PR_ERR_ARG, "lr_off not monotone");
    const int64_t l_pac = n_lr ? lr_off[n_lr] - lr_off[0] : 0;
    if (2 * l_pac + 2 * (int64_t)n_lr > seedc::MAX_TEXT)
        return set_error(PR_ERR_CAPACITY, "long reads beyond the index's 2^33 text positions (l_pac < 4.29 Gb)");
    if ((int64_t)n_lr >= ((int64_t)1 << seedc::FR_RID_BITS))
        return set_error(PR_ERR_CAPACITY, "more than 2^24 long reads in one index");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    DevBuf *D = c->sd;
    const int64_t n_text = 2 * l_pac + 2 * (int64_t)n_lr;
    // small host tables: rebased read offsets, contig starts, 4 KB block -> contig
    std::vector<int64_t> off((size_t)n_lr + 1, 0), cstart(2 * (size_t)n_lr, 0);
    for (int i = 0; i <= n_lr; ++i) off[(size_t)i] = lr_off[i] - (n_lr ? lr_off[0] : 0);
    for (int i = 0; i < n_lr; ++i) {
        cstart[(size_t)i] = off[(size_t)i] + i;
        cstart[2 * (size_t)n_lr - 1 - i] = l_pac + n_lr + (l_pac - off[(size_t)i + 1]) + (n_lr - 1 - i);
    }
    const int64_t nb = (n_text >> seedc::CB_SHIFT) + 1;
    std::vector<int32_t> cblk((size_t)nb, 0);
    {
        int ci = 0;
        const int nc = 2 * n_lr;
        for (int64_t b = 0; b < nb; ++b) {
            while (ci + 1 < nc && cstart[(size_t)ci + 1] <= (b << seedc::CB_SHIFT)) ++ci;
            cblk[(size_t)b] = ci;
        }
    }
    const size_t nt = (size_t)(n_text > 0 ? n_text : 1);
    // sorts of up to 2^31 text positions when the device has room for their buffers (~16 bytes a
    // position + rocPRIM's temporaries: configs[2]'s 2.1 G-position text in one sort, 293 -> 151
    // ms), else 2^30 (a divisor of 2^32 either way; PRGPU_INDEX_CHUNK=k: 2^k, a test hook that
    // sends small texts through the chunked build)
    int64_t chunk = (int64_t)1 << 30;
    if (n_text > chunk) {
        size_t fr = 0, tot = 0;
        (void)hipMemGetInfo(&fr, &tot);
        (void)hipGetLastError();
        const int64_t have = (int64_t)(D[SX_KEY0].cap + D[SX_KEY1].cap + D[SX_VAL0].cap + D[SX_VAL1].cap + D[SX_TEMP].cap);
        // (room for the bigger sort buffers with 64 GB to spare for the rest of the task)
        if ((int64_t)fr + have >= ((int64_t)1 << 31) * 20 + ((int64_t)64 << 30)) chunk = (int64_t)1 << 31;
    }
    if (const char *ch = getenv("PRGPU_INDEX_CHUNK")) {
        const int k = atoi(ch);
        if (k >= 16 && k <= 31) chunk = (int64_t)1 << k;
    }
    const bool chunked = n_text > chunk;
    const size_t ns = (size_t)(chunked ? chunk : (int64_t)nt);   // sort scratch entries
    const size_t temp = seed_index_temp_bytes((int64_t)ns);
    const size_t nk1 = (size_t)seedc::NK + 1;
    // hits <= 12-mer starts; kpos / kext sized by the text (the count is known after the build)
    int rc;
    if ((rc = upload(D[SX_LRSEQ], lr_dev ? nullptr : (n_lr ? lr_seq + lr_off[0] : lr_seq), (size_t)l_pac, s)) ||
        (rc = upload(D[SI_LROFF], off.data(), off.size(), s)) || (rc = upload(D[SI_CSTART], cstart.data(), cstart.size(), s)) ||
        (rc = upload(D[SI_CBLK], cblk.data(), cblk.size(), s)) || (rc = D[SI_TEXT].ensure(nt)) ||
        (rc = D[SX_KEY0].ensure(ns * 4)) || (rc = D[SX_KEY1].ensure(ns * 4)) || (rc = D[SX_VAL0].ensure(ns * 4)) ||
        (rc = D[SX_KC].ensure(nk1 * 4)) || (rc = D[SI_KOFF].ensure(nk1 * 8)) ||
        (rc = D[SI_KPOS].ensure(nt * 4)) || (rc = D[SI_KEXT].ensure(nt * 8)) || (rc = D[SX_TEMP].ensure(temp)) ||
        (rc = D[SX_CNTPTR].ensure(sizeof(uint32_t *) * (seedc::KI - 1))))
        return rc;
    if (chunked && ((rc = D[SX_VAL1].ensure(ns * 4)) || (rc = D[SX_KCC].ensure(nk1 * 4)) ||
                    (rc = D[SX_KOFFC].ensure(nk1 * 4)) || (rc = D[SX_KCUR].ensure(nk1 * 8))))
        return rc;
    const bool paged = n_text > (int64_t)seedc::POS_PAGE;
    if (paged && (rc = D[SI_KSPLIT].ensure(nk1 * 8))) return rc;
    if (lr_dev && l_pac) HIPCHK(hipMemcpyAsync(D[SX_LRSEQ].p, lr_seq + lr_off[0], (size_t)l_pac, hipMemcpyDeviceToDevice, s));
    SeedIndexBuild B{};
    uint32_t *cptr[seedc::KI - 1];
    for (int j = 1; j < seedc::KI; ++j) {
        if ((rc = D[SI_CNT0 + j - 1].ensure(((size_t)1 << (2 * j)) * 4))) return rc;
        cptr[j - 1] = B.cnt[j - 1] = D[SI_CNT0 + j - 1].as<uint32_t>();
    }
    HIPCHK(hipMemcpyAsync(D[SX_CNTPTR].p, cptr, sizeof cptr, hipMemcpyHostToDevice, s));
    B.lr_seq = D[SX_LRSEQ].as<uint8_t>();
    B.lr_off = D[SI_LROFF].as<int64_t>();
    B.n_lr = n_lr;
    B.l_pac = l_pac;
    B.cstart = D[SI_CSTART].as<int64_t>();
    B.n_text = n_text;
    B.text = D[SI_TEXT].as<uint8_t>();
    B.chunk = chunk;
    B.key0 = D[SX_KEY0].as<uint32_t>();
    B.key1 = D[SX_KEY1].as<uint32_t>();
    B.val0 = D[SX_VAL0].as<uint32_t>();
    B.val1 = chunked ? D[SX_VAL1].as<uint32_t>() : nullptr;
    B.kc = D[SX_KC].as<uint32_t>();
    B.koff = D[SI_KOFF].as<uint64_t>();
    B.kcc = chunked ? D[SX_KCC].as<uint32_t>() : nullptr;
    B.koffc = chunked ? D[SX_KOFFC].as<uint32_t>() : nullptr;
    B.kcur = chunked ? D[SX_KCUR].as<uint64_t>() : nullptr;
    B.kpos = D[SI_KPOS].as<uint32_t>();
    B.kext = D[SI_KEXT].as<uint64_t>();
    B.ksplit = paged ? D[SI_KSPLIT].as<uint64_t>() : nullptr;
    B.cnt_dev = reinterpret_cast<uint32_t *const *>(D[SX_CNTPTR].p);
    B.temp = D[SX_TEMP].p;
    B.temp_bytes = temp;
    HIPCHK(hipEventRecord(c->ev[8], s));
    const int e = seed_index_device_build(B, s);
    if (e) return set_error(PR_ERR_HIP, "seed index build: %s", hipGetErrorString((hipError_t)e));
    HIPCHK(hipEventRecord(c->ev[9], s));
    uint64_t nh = 0;
    HIPCHK(hipMemcpyAsync(&nh, B.koff + seedc::NK, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->ev[8], c->ev[9]) == hipSuccess) c->ms_index = ms;
    if (n_text > (int64_t)seedc::POS_PAGE) {
        // a build beyond 2^32 positions (configs[3] ranks) gives its sort buffers back (4 x 4-8 GB +
        // rocPRIM's temporaries): there a rank's device memory peaks near the card's 288 GiB later
        // in the task (DESIGN.md current status); smaller texts keep them for the next task's
        // build (no re-allocation inside a timed step)
        for (int id : {(int)SX_KEY0, (int)SX_KEY1, (int)SX_VAL0, (int)SX_VAL1, (int)SX_TEMP}) D[id].release();
    }
    seedc::IndexView v{};
    v.text = B.text;
    v.n_text = n_text;
    v.cstart = B.cstart;
    v.n_contig = 2 * n_lr;
    v.cblk = D[SI_CBLK].as<int32_t>();
    v.lr_off = B.lr_off;
    v.n_lr = n_lr;
    v.l_pac = l_pac;
    v.koff = B.koff;
    v.kpos = B.kpos;
    v.kext = B.kext;
    v.ksplit = B.ksplit;
    for (int j = 0; j < seedc::KI - 1; ++j) v.cnt[j] = B.cnt[j];
    if ((rc = seed_text4(c, v, s))) return rc;
    if ((rc = upload_blk_fr(c, v, cstart.data(), off.data(), n_lr, l_pac, n_text, s))) return rc;
    c->seed_view = v;
    c->seed_loaded = true;
    c->seed_n_text = n_text;
    c->seed_n_hits = nh;
    return 0;
}

// the six digests of pr_seed_index_digest over the device index (test hook)
extern "C" int pr_seed_gpu_index_digest(pr_ctx *c, uint64_t *out6) {
    if (!c || !out6) return set_error(PR_ERR_ARG, "null arg");
    if (!c->seed_loaded || !c->seed_n_text) return set_error(PR_ERR_ARG, "no device-built seed index");
    HIPCHK(hipSetDevice(c->device));
    const seedc::IndexView &v = c->seed_view;
    const size_t nt = (size_t)c->seed_n_text, nh = (size_t)c->seed_n_hits, nk = (size_t)seedc::NK;
    std::vector<uint8_t> text(nt);
    std::vector<uint64_t> koff(nk + 1);
    std::vector<uint32_t> kpos(nh), kc(nk);
    std::vector<uint64_t> kext(nh);
    std::vector<int64_t> cstart((size_t)v.n_contig), lro((size_t)v.n_lr + 1);
    std::vector<int32_t> cblk((size_t)((c->seed_n_text >> seedc::CB_SHIFT) + 1));
    std::vector<std::vector<uint32_t>> cnt(seedc::KI);
    HIPCHK(hipMemcpy(text.data(), v.text, nt, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(koff.data(), v.koff, (nk + 1) * 8, hipMemcpyDeviceToHost));
    if (nh) HIPCHK(hipMemcpy(kpos.data(), v.kpos, nh * 4, hipMemcpyDeviceToHost));
    if (nh) HIPCHK(hipMemcpy(kext.data(), v.kext, nh * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(kc.data(), c->sd[SX_KC].p, nk * 4, hipMemcpyDeviceToHost));
    if (!cstart.empty()) HIPCHK(hipMemcpy(cstart.data(), v.cstart, cstart.size() * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(lro.data(), v.lr_off, lro.size() * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cblk.data(), v.cblk, cblk.size() * 4, hipMemcpyDeviceToHost));
    for (int j = 0; j < seedc::KI - 1; ++j) {
        cnt[(size_t)j].resize((size_t)1 << (2 * (j + 1)));
        HIPCHK(hipMemcpy(cnt[(size_t)j].data(), v.cnt[j], cnt[(size_t)j].size() * 4, hipMemcpyDeviceToHost));
    }
    cnt[seedc::KI - 1] = std::move(kc);
    std::vector<uint64_t> ksplit(v.ksplit ? nk : 0);
    if (v.ksplit) HIPCHK(hipMemcpy(ksplit.data(), v.ksplit, nk * 8, hipMemcpyDeviceToHost));
    seed_digest_tables(text, koff, kpos, kext, cnt, cstart, cblk, lro, ksplit, out6);
    return 0;
}

extern "C" int pr_seed_gpu_index_koff(pr_ctx *c, uint64_t *koff, uint64_t *ksplit) {
    if (!c || !koff) return set_error(PR_ERR_ARG, "null arg");
    if (!c->seed_loaded) return set_error(PR_ERR_ARG, "no device seed index");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(koff, c->seed_view.koff, ((size_t)seedc::NK + 1) * 8, hipMemcpyDeviceToHost));
    if (ksplit && c->seed_view.ksplit)
        HIPCHK(hipMemcpy(ksplit, c->seed_view.ksplit, (size_t)seedc::NK * 8, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int pr_seed_gpu_index_last_ms(pr_ctx *c, double *ms) {
    if (!c || !ms) return set_error(PR_ERR_ARG, "null arg");
    *ms = c->ms_index;
    return 0;
}

// the resident short reads (include/prgpu.h pr_srset_load): the whole short-read input once;
// a task's sample is gathered on the device from its record ranges
extern "C" int pr_srset_load(pr_ctx *c, int64_t n_sr, const int64_t *off, const uint8_t *seq) {
    if (!c || n_sr < 0 || !off || (off[n_sr] && !seq) || off[0] != 0) return set_error(PR_ERR_ARG, "bad arg");
    HIPCHK(hipSetDevice(c->device));
    int rc = upload(c->ls[LS_SRSEQ], seq, (size_t)off[n_sr], c->stream);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    c->ss_off.assign(off, off + n_sr + 1);
    c->ss_samp_off.clear();
    c->ls[LS_SRSAMP].release();
    return 0;
}

extern "C" int pr_srset_sample(pr_ctx *c, const int64_t *ranges, int n_ranges) {
    if (!c || n_ranges < 0 || (n_ranges && !ranges)) return set_error(PR_ERR_ARG, "null arg");
    if (c->ss_off.empty()) return set_error(PR_ERR_ARG, "no resident short reads (pr_srset_load)");
    const int64_t N = (int64_t)c->ss_off.size() - 1;
    std::vector<int64_t> off(1, 0);
    for (int k = 0; k < n_ranges; ++k) {
        const int64_t r0 = ranges[2 * k], r1 = ranges[2 * k + 1];
        if (r0 < 0 || r1 < r0 || r1 > N) return set_error(PR_ERR_ARG, "record range outside the short reads");
        for (int64_t i = r0; i < r1; ++i) off.push_back(off.back() + c->ss_off[(size_t)i + 1] - c->ss_off[(size_t)i]);
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc = c->ls[LS_SRSAMP].ensure((size_t)off.back() + 1);
    if (rc) return rc;
    int64_t at = 0;
    for (int k = 0; k < n_ranges; ++k) {
        const int64_t b0 = c->ss_off[(size_t)ranges[2 * k]], b1 = c->ss_off[(size_t)ranges[2 * k + 1]];
        if (b1 > b0)
            HIPCHK(hipMemcpyAsync(c->ls[LS_SRSAMP].as<uint8_t>() + at, c->ls[LS_SRSEQ].as<uint8_t>() + b0, (size_t)(b1 - b0),
                                  hipMemcpyDeviceToDevice, s));
        at += b1 - b0;
    }
    c->ss_samp_off.swap(off);
    return 0;
}

extern "C" int pr_seed_gpu_map_sampled(pr_ctx *c, const pr_seed_opts *o, const int64_t *ranges, int n_ranges,
                                       int32_t *status) {
    if (!c || !o || n_ranges < 0 || (n_ranges && !ranges)) return set_error(PR_ERR_ARG, "null arg");
    if (c->ss_off.empty()) return set_error(PR_ERR_ARG, "no resident short reads (pr_srset_load)");
    const int64_t N = (int64_t)c->ss_off.size() - 1;
    std::vector<int64_t> off(1, 0);
    for (int k = 0; k < n_ranges; ++k) {
        const int64_t r0 = ranges[2 * k], r1 = ranges[2 * k + 1];
        if (r0 < 0 || r1 < r0 || r1 > N) return set_error(PR_ERR_ARG, "record range outside the short reads");
        for (int64_t i = r0; i < r1; ++i) off.push_back(off.back() + c->ss_off[(size_t)i + 1] - c->ss_off[(size_t)i]);
    }
    const int64_t n = (int64_t)off.size() - 1;
    if (n > INT32_MAX) return set_error(PR_ERR_CAPACITY, "too many short reads in one sample");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc = c->sd[SB_SEQ].ensure((size_t)off.back() + 1);
    if (rc) return rc;
    int64_t at = 0;
    for (int k = 0; k < n_ranges; ++k) {
        const int64_t b0 = c->ss_off[(size_t)ranges[2 * k]], b1 = c->ss_off[(size_t)ranges[2 * k + 1]];
        if (b1 > b0)
            HIPCHK(hipMemcpyAsync(c->sd[SB_SEQ].as<uint8_t>() + at, c->ls[LS_SRSEQ].as<uint8_t>() + b0, (size_t)(b1 - b0),
                                  hipMemcpyDeviceToDevice, s));
        at += b1 - b0;
    }
    c->seed_sr_staged = true;
    return pr_seed_gpu_map(c, o, nullptr, off.data(), (int)n, nullptr, status);
}

extern "C" int pr_seed_gpu_map(pr_ctx *c, const pr_seed_opts *o, const uint8_t *sr_seq, const int64_t *sr_off, int n_sr,
                               pr_seed_tasks *out, int32_t *status) {
    if (!c) return set_error(PR_ERR_ARG, "null arg");
    const bool staged = c->seed_sr_staged;   // pr_seed_gpu_map_sampled gathered the reads on the device
    c->seed_sr_staged = false;
    if (!o || n_sr < 0 || (n_sr && ((!sr_seq && !staged) || !sr_off))) return set_error(PR_ERR_ARG, "null arg");
    pr_seed_tasks dummy;
    const bool keep_on_device = out == nullptr;
    if (!out) out = &dummy;
    c->seed_pre.clear();
    if (!c->seed_loaded) return set_error(PR_ERR_ARG, "no seed index on the device (pr_seed_gpu_upload)");
    if (o->min_seed_len < seedc::KI) return set_error(PR_ERR_UNSUPPORTED, "min seed length below the 12-mer index");
    if (o->max_occ <= 0 || o->w < 0) return set_error(PR_ERR_ARG, "bad seeding options");
    out->n = 0;
    out->t = nullptr;
    if (n_sr && sr_off[0] != 0) return set_error(PR_ERR_ARG, "sr_off must start at 0");
    for (int i = 0; i < n_sr; ++i)
        if (sr_off[i + 1] < sr_off[i]) return set_error(PR_ERR_ARG, "sr_off not monotone");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    DevBuf *D = c->sd;
    int qmax = 1;
    for (int i = 0; i < n_sr; ++i) qmax = std::max<int>(qmax, (int)(sr_off[i + 1] - sr_off[i]));
    seedc::Caps caps = seedc::device_caps(qmax);
    caps.hi = c->seed_view.ksplit != nullptr;   // text beyond 2^32: positions carry bit 32
    caps.nopos = 1;   // the device tables keep the chaining's coordinates only (seed_core.h Caps)
    // pass 1: 64 reads per wave, small slices sized for the batch; pass 2 (flagged reads): the
    // large slices, one wave per read
    seedc::Caps small = seedc::device_caps_small(std::min(qmax, caps.lmax));
    small.hi = caps.hi;
    small.nopos = 1;
    // the finish tasks' near-exact mapping: pass 1's occurrence tables lazily, a start's hits on
    // first use (seed_core.h materialize; the later passes build them eagerly, wave-parallel)
    small.lazy = seedc::lazy_occ(*o) ? 1 : 0;
    if (const char *sc = getenv("PRGPU_SEED_SMALL"))   // tuning hook: hits,iv,mems,seeds,chains
        sscanf(sc, "%d,%d,%d,%d,%d", &small.hits, &small.iv, &small.mems, &small.seeds, &small.chains);
    SeedDev K{};
    K.V = c->seed_view;
    K.O = *o;
    K.n_sr = n_sr;
    K.caps = small;
    K.stride = seedc::scratch_bytes(small);
    const char *wpc = getenv("PRGPU_SEED_WAVES_PER_CU");   // tuning hook
    int64_t waves = (int64_t)c->n_cu * (wpc ? atoi(wpc) : 16);   // ~98 KB x 64 slices per wave at 150 bp
    const int64_t nbatch = (n_sr + 63) / 64;
    if (waves > nbatch) waves = nbatch;
    if (waves < 1) waves = 1;
    // PRGPU_SEED_BALANCE: every wave the same number of 64-read batches (fewer waves; measured
    // slower at configs[1], 357 vs 345 ms: the lane phase wants every wave it can get)
    if (getenv("PRGPU_SEED_BALANCE")) {
        const int64_t rounds = (nbatch + waves - 1) / waves;
        waves = (nbatch + rounds - 1) / rounds;
    }
    {   // pass 1's slices within a scratch budget: 15 % of the free device memory, between 24 and
        // 40 GB (configs[1]'s 16 waves per CU need ~32 GB; long mr reads: fewer waves).  (Round 4
        // capped it at 24 GB, which cut configs[1] to ~3,800 of its 4,096 waves.)
        size_t fr = 0, tot = 0;
        (void)hipMemGetInfo(&fr, &tot);
        (void)hipGetLastError();
        const int64_t have = (int64_t)D[SB_SCRATCH].cap;   // (already ours: counts as free)
        const int64_t budget = std::min<int64_t>((int64_t)40 << 30,
                                                 std::max<int64_t>((int64_t)24 << 30, ((int64_t)fr + have) * 15 / 100));
        const int64_t wmax = std::max<int64_t>(c->n_cu, budget / (64 * K.stride));
        if (waves > wmax) waves = wmax;
    }
    K.n_lanes = waves;
    // mem_flt_chained_seeds' SW rows of pass 1 (reads >= 440 bp), lane-interleaved per wave
    K.dp = nullptr;
    if (seedc::seed_flt_min_score(*o, qmax) >= 0) {
        int rc0 = D[SB_DP].ensure((size_t)waves * 2 * 201 * 64 * sizeof(int16_t));
        if (rc0) return rc0;
        K.dp = D[SB_DP].as<int16_t>();
    }
    int64_t lanes2 = (int64_t)c->n_cu * seed_slots_per_cu(c->seed_view.walk_nw);
    const int64_t scratch = std::max<int64_t>(waves * 64 * K.stride, lanes2 * seedc::scratch_bytes(caps));
    const int64_t nb = n_sr ? sr_off[n_sr] : 0;
    // reads are mapped in chunks whose output slabs (caps.out seeds per read) fit a budget
    // (PRGPU_SEED_OUT_MB, default 8 GB; configs[1]'s 460k reads are one chunk); every chunk's
    // seeds are compacted into the dense list before the next chunk reuses the slab
    const int64_t slot_bytes = (int64_t)caps.out * (int64_t)sizeof(pr_seed_task);
    const char *ob = getenv("PRGPU_SEED_OUT_MB");
    const int64_t out_budget = (ob ? std::max<int64_t>(1, atoll(ob)) : 8192) << 20;
    const int64_t chunk = std::max<int64_t>(64, out_budget / slot_bytes / 64 * 64);
    int rc;
    c->seed_sr_bases = nb;
    if ((!staged && (rc = upload(D[SB_SEQ], sr_seq, (size_t)nb, s))) || (rc = upload(D[SB_OFF], sr_off, (size_t)n_sr + 1, s)) ||
        (rc = D[SB_SCRATCH].ensure((size_t)scratch)) ||
        (rc = D[SB_OUT].ensure((size_t)(std::min<int64_t>(chunk, n_sr) * slot_bytes + 16))) ||
        (rc = D[SB_NOUT].ensure((size_t)n_sr * 4 + 16)) || (rc = D[SB_STATUS].ensure((size_t)n_sr * 4 + 16)) ||
        (rc = D[SB_NEXT].ensure(256)) || (rc = D[SB_PRE].ensure(((size_t)n_sr + 1) * 8)) ||
        (rc = D[SB_DENSE].ensure(sizeof(pr_seed_task))))
        return rc;
    K.sr_seq = D[SB_SEQ].as<uint8_t>();
    K.sr_off = D[SB_OFF].as<int64_t>();
    K.out = D[SB_OUT].as<pr_seed_task>();
    K.n_out = D[SB_NOUT].as<int32_t>();
    K.status = D[SB_STATUS].as<int32_t>();
    K.next = D[SB_NEXT].as<int32_t>();
    K.prof = reinterpret_cast<unsigned long long *>(D[SB_NEXT].as<uint8_t>() + 64);
    HIPCHK(hipMemsetAsync(K.next, 0, 256, s));
    HIPCHK(hipEventRecord(c->ev[8], s));
    c->seed_pass2 = 0;
    c->seed_pass3 = 0;
    std::vector<int32_t> nout((size_t)n_sr), st((size_t)n_sr);
    std::vector<int64_t> pre((size_t)n_sr + 1, 0);
    int64_t total = 0, bad = 0;
    int32_t bad_flags = 0;
    for (int64_t r0 = 0; r0 < n_sr; r0 += chunk) {
        const int64_t r1 = std::min<int64_t>(n_sr, r0 + chunk);
        K.caps = small;
        K.stride = seedc::scratch_bytes(small);
        K.n_lanes = waves;
        K.scratch = D[SB_SCRATCH].as<uint8_t>();
        K.rlist = nullptr;
        K.n_list = 0;
        K.out0 = r0;
        K.n_sr = r1;
        int32_t start = (int32_t)r0;
        // PRGPU_SEED_LPT=1: the chunk's reads costliest first (seed_order_launch).  Measured at
        // configs[1]: 312.5 against 306.2 ms in read order (the batches' lane phase grew more than
        // the tail shrank), so read order stays the default
        const char *lpt = getenv("PRGPU_SEED_LPT");
        if (lpt && lpt[0] == '1') {
            int32_t *order = nullptr;
            if ((rc = D[SB_ORDER].ensure(seed_order_bytes(r1 - r0)))) return rc;
            int eo = seed_order_launch(K, r0, r1 - r0, D[SB_ORDER].p, &order, (void *)s);
            if (eo) return set_error(PR_ERR_HIP, "seed order: %s", hipGetErrorString((hipError_t)eo));
            K.rlist = order;
            K.n_list = r1 - r0;
            start = 0;
        }
        HIPCHK(hipMemcpyAsync(K.next, &start, 4, hipMemcpyHostToDevice, s));
        int e = seed_batch_launch(K, (void *)s);
        if (e) return set_error(PR_ERR_HIP, "seed kernel: %s", hipGetErrorString((hipError_t)e));
        if (r0 == 0) HIPCHK(hipEventRecord(c->ev[10], s));
        std::vector<int32_t> st1((size_t)(r1 - r0)), no1((size_t)(r1 - r0));
        if ((rc = download(st1.data(), D[SB_STATUS], (size_t)(r1 - r0), s, (size_t)r0)) ||
            (rc = download(no1.data(), D[SB_NOUT], (size_t)(r1 - r0), s, (size_t)r0)))
            return rc;
        HIPCHK(hipStreamSynchronize(s));
        std::vector<int32_t> redo;
        // pass 2's slices; after the by-wave pass 1b they are that pass's (its leftovers overflowed
        // them), so pass 2 is skipped and the later passes grow from them
        seedc::Caps p2caps = caps;
        bool p2_ran = false;
        int32_t fl1 = 0;
        int64_t need_hits = 0;   // the largest hit table a flagged read asked for
        int64_t need_sum = 0, need_n = 0;   // (and their mean)
        for (int64_t i = r0; i < r1; ++i)
            if (st1[(size_t)(i - r0)]) {
                redo.push_back((int32_t)i);
                fl1 |= st1[(size_t)(i - r0)];
                need_hits = std::max<int64_t>(need_hits, -(int64_t)no1[(size_t)(i - r0)]);
                if (no1[(size_t)(i - r0)] < 0) need_sum -= no1[(size_t)(i - r0)], ++need_n;
            }
        // many flagged reads (the finish task maps to corrected reads at 30x long-read coverage:
        // ~140 starts x 30 hits > 4096 for nearly every read): pass 1 again, lane per read, over
        // them with the arrays that overflowed grown (within the scratch already allocated),
        // instead of pass 2's one wave per read
        if (redo.size() > 4096 && !(fl1 & (seedc::SC_OVER_LEN | seedc::SC_OVER_OUT))) {
            seedc::Caps cb = small;
            // the hit tables sized for the largest flagged read (dense indexes: configs[2] /
            // configs[3], or N > 1 ranks of the exact layout, every read overflows pass 1)
            if (fl1 & seedc::SC_OVER_HITS) {
                // the largest flagged read's hit table (+ 1/8), not a multiple of pass 1's: the finish
                // task's reads need just over pass 1's 4096 hits, and 4x slices cut the waves in flight
                // (the occurrence table is latency-bound: 413 -> measured in DESIGN.md §5 round 6)
                cb.hits = (int32_t)std::min<int64_t>(std::max<int64_t>((int64_t)cb.hits + 512, (need_hits + need_hits / 8 + 511) & ~(int64_t)511),
                                                     (int64_t)1 << 20);
                // their chaining never ran; random 12-mer hits become chains and seeds in
                // proportion to the hits, so those arrays grow by the same factor
                const int64_t f = std::min<int64_t>(16, std::max<int64_t>(1, cb.hits / small.hits));
                cb.chains = (int32_t)(cb.chains * f);
                cb.seeds = (int32_t)(cb.seeds * f);
            }
            if (fl1 & seedc::SC_OVER_IV) cb.iv *= 2;
            if (fl1 & seedc::SC_OVER_MEMS) cb.mems *= 2;
            if (fl1 & seedc::SC_OVER_SEEDS) cb.seeds *= 2;
            if (fl1 & seedc::SC_OVER_CHAINS) cb.chains *= 2;
            const int64_t sb = seedc::scratch_bytes(cb);
            {   // room for as many waves as pass 1 ran (or the flagged reads' batches), within pass 1's budget
                size_t fr = 0, tot = 0;
                (void)hipMemGetInfo(&fr, &tot);
                (void)hipGetLastError();
                const int64_t have = (int64_t)D[SB_SCRATCH].cap;
                const int64_t budget = std::min<int64_t>((int64_t)40 << 30,
                                                         std::max<int64_t>((int64_t)24 << 30, ((int64_t)fr + have) * 15 / 100));
                const int64_t want = std::min<int64_t>(waves, ((int64_t)redo.size() + 63) / 64) * 64 * sb;
                if (want > have && want <= budget) {
                    HIPCHK(hipStreamSynchronize(s));
                    if ((rc = D[SB_SCRATCH].ensure((size_t)want))) return rc;
                    K.scratch = D[SB_SCRATCH].as<uint8_t>();
                }
            }
            int64_t wb = std::min<int64_t>((int64_t)D[SB_SCRATCH].cap / (64 * sb), ((int64_t)redo.size() + 63) / 64);
            wb = std::min<int64_t>(wb, waves);   // (the filter rows' area holds `waves` waves)
            // reads that need more than 4x pass 1's hits on average (dense indexes: configs[2] / [3]) one wave
            // each (seed_wave_kernel: the chaining over the lanes) with pass 2's slices grown like
            // cb: 64 such slices per wave fit only a few hundred waves in the scratch (a configs[3]
            // rank's seeding 17.4 -> 4.1 s, configs[2] 1.01 -> 0.82 s).  The finish task's reads
            // (just over pass 1's hits, ~30x coverage) stay lane per read (620 vs 724 ms as waves).
            // PRGPU_SEED_1B=wave / lane forces either.
            const char *p1b = getenv("PRGPU_SEED_1B");
            const bool by_wave = p1b ? !strcmp(p1b, "wave") : need_sum > 4 * (int64_t)small.hits * need_n;
            seedc::Caps cw = caps;
            cw.hits = std::max(caps.hits, cb.hits);
            cw.iv = std::max(caps.iv, cb.iv);
            cw.mems = std::max(caps.mems, cb.mems);
            cw.seeds = std::max(caps.seeds, cb.seeds);
            cw.chains = std::max(caps.chains, cb.chains);
            const int64_t sw = seedc::scratch_bytes(cw);
            const int64_t ww = std::min<int64_t>(std::min<int64_t>(lanes2, (int64_t)redo.size()), (int64_t)D[SB_SCRATCH].cap / sw);
            if (by_wave && ww >= c->n_cu) {
                K.caps = cw;
                K.stride = sw;
                K.n_lanes = ww;
                K.rlist = D[SB_PRE].as<int32_t>();
                K.n_list = (int64_t)redo.size();
                HIPCHK(hipMemcpyAsync(D[SB_PRE].p, redo.data(), redo.size() * 4, hipMemcpyHostToDevice, s));
                HIPCHK(hipMemsetAsync(K.next, 0, 4, s));
                e = seed_launch(K, (void *)s);
                if (e) return set_error(PR_ERR_HIP, "seed kernel (pass 1b, waves): %s", hipGetErrorString((hipError_t)e));
                p2caps = cw;
                p2_ran = true;
                std::vector<int32_t> st1b((size_t)(r1 - r0));
                if ((rc = download(st1b.data(), D[SB_STATUS], (size_t)(r1 - r0), s, (size_t)r0))) return rc;
                HIPCHK(hipStreamSynchronize(s));
                std::vector<int32_t> left;
                for (int32_t i : redo)
                    if (st1b[(size_t)(i - r0)]) left.push_back(i);
                redo.swap(left);
                K.rlist = nullptr;
                K.n_list = 0;
            } else if (wb >= c->n_cu) {
                K.caps = cb;
                K.stride = sb;
                K.n_lanes = wb;
                K.rlist = D[SB_PRE].as<int32_t>();
                K.n_list = (int64_t)redo.size();
                HIPCHK(hipMemcpyAsync(D[SB_PRE].p, redo.data(), redo.size() * 4, hipMemcpyHostToDevice, s));
                HIPCHK(hipMemsetAsync(K.next, 0, 4, s));
                e = seed_batch_launch(K, (void *)s);
                if (e) return set_error(PR_ERR_HIP, "seed kernel (pass 1b): %s", hipGetErrorString((hipError_t)e));
                std::vector<int32_t> st1b((size_t)(r1 - r0));
                if ((rc = download(st1b.data(), D[SB_STATUS], (size_t)(r1 - r0), s, (size_t)r0))) return rc;
                HIPCHK(hipStreamSynchronize(s));
                std::vector<int32_t> left;
                for (int32_t i : redo)
                    if (st1b[(size_t)(i - r0)]) left.push_back(i);
                redo.swap(left);
                K.rlist = nullptr;
                K.n_list = 0;
            }
        }
        c->seed_pass2 += (int64_t)redo.size();
        if (!redo.empty()) {   // pass 2 over the flagged reads (rlist in SB_PRE)
            K.rlist = D[SB_PRE].as<int32_t>();
            if (!p2_ran) {
                HIPCHK(hipMemcpyAsync(D[SB_PRE].p, redo.data(), redo.size() * 4, hipMemcpyHostToDevice, s));
                HIPCHK(hipMemsetAsync(K.next, 0, 4, s));
                K.caps = caps;
                K.stride = seedc::scratch_bytes(caps);
                K.n_lanes = std::min<int64_t>(lanes2, (int64_t)redo.size());
                K.n_list = (int64_t)redo.size();
                e = seed_launch(K, (void *)s);
                if (e) return set_error(PR_ERR_HIP, "seed kernel (pass 2): %s", hipGetErrorString((hipError_t)e));
                HIPCHK(hipStreamSynchronize(s));
            }
            // later passes: the reads that outgrew the large slices too (e.g. the finish task's
            // near-exact reads at 30-60x long-read coverage: every 12-mer hits every copy, > 8192
            // hits per read) again, with the arrays that overflowed grown, up to 4 times
            seedc::Caps cg = p2caps;
            for (int pass = 3; pass <= 6; ++pass) {
                std::vector<int32_t> st2((size_t)(r1 - r0));
                if ((rc = download(st2.data(), D[SB_STATUS], (size_t)(r1 - r0), s, (size_t)r0))) return rc;
                HIPCHK(hipStreamSynchronize(s));
                std::vector<int32_t> again;
                int32_t fl = 0;
                for (int32_t i : redo)
                    if (st2[(size_t)(i - r0)]) again.push_back(i), fl |= st2[(size_t)(i - r0)];
                if (again.empty() || (fl & (seedc::SC_OVER_LEN | seedc::SC_OVER_OUT))) break;
                if (fl & seedc::SC_OVER_HITS) cg.hits *= 4;
                if (fl & seedc::SC_OVER_IV) cg.iv *= 2;
                if (fl & seedc::SC_OVER_MEMS) cg.mems *= 2;
                if (fl & seedc::SC_OVER_SEEDS) cg.seeds *= 2;
                if (fl & seedc::SC_OVER_CHAINS) cg.chains *= 2;
                redo.swap(again);
                K.caps = cg;
                K.stride = seedc::scratch_bytes(cg);
                K.n_lanes = std::min<int64_t>(lanes2, (int64_t)redo.size());
                if ((rc = D[SB_SCRATCH].ensure((size_t)(K.n_lanes * K.stride)))) return rc;
                K.scratch = D[SB_SCRATCH].as<uint8_t>();
                K.n_list = (int64_t)redo.size();
                HIPCHK(hipMemcpyAsync(D[SB_PRE].p, redo.data(), redo.size() * 4, hipMemcpyHostToDevice, s));
                HIPCHK(hipMemsetAsync(K.next, 0, 4, s));
                e = seed_launch(K, (void *)s);
                if (e) return set_error(PR_ERR_HIP, "seed kernel (pass %d): %s", pass, hipGetErrorString((hipError_t)e));
                HIPCHK(hipStreamSynchronize(s));
                c->seed_pass3 += (int64_t)redo.size();
            }
        }
        // the chunk's seeds: compacted on the device (read order) behind the earlier chunks'
        if ((rc = download(nout.data() + r0, D[SB_NOUT], (size_t)(r1 - r0), s, (size_t)r0)) ||
            (rc = download(st.data() + r0, D[SB_STATUS], (size_t)(r1 - r0), s, (size_t)r0)))
            return rc;
        HIPCHK(hipStreamSynchronize(s));
        const int64_t t0 = total;
        for (int64_t i = r0; i < r1; ++i) {
            if (nout[(size_t)i] < 0 || nout[(size_t)i] > caps.out) return set_error(PR_ERR_HIP, "seed kernel: bad task count");
            total += nout[(size_t)i];
            pre[(size_t)i + 1] = total;
            bad += st[(size_t)i] != 0;
            bad_flags |= st[(size_t)i];
        }
        if ((rc = upload(D[SB_PRE], pre.data() + r0, (size_t)(r1 - r0 + 1), s)) ||
            (rc = D[SB_DENSE].grow_keep(sizeof(pr_seed_task) * (size_t)(total > 0 ? total : 1),
                                        sizeof(pr_seed_task) * (size_t)t0, s)))
            return rc;
        const int e2 = seed_compact_launch(D[SB_OUT].as<pr_seed_task>(), D[SB_NOUT].as<int32_t>() + r0,
                                           D[SB_PRE].as<int64_t>(), r1 - r0, caps.out, D[SB_DENSE].as<pr_seed_task>(),
                                           (void *)s);
        if (e2) return set_error(PR_ERR_HIP, "seed compaction: %s", hipGetErrorString((hipError_t)e2));
    }
    HIPCHK(hipEventRecord(c->ev[9], s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0.f;
    if (n_sr && hipEventElapsedTime(&ms, c->ev[8], c->ev[9]) == hipSuccess) c->ms_seed = ms;
    c->ms_seed_pass2 = 0.f;   // (the passes after the first chunk's pass 1; one chunk at configs[1])
    if (n_sr && hipEventElapsedTime(&ms, c->ev[10], c->ev[9]) == hipSuccess) c->ms_seed_pass2 = ms;

    // an incomplete seed set (flagged reads have no seeds) is never handed to
    // pr_iter_upload_gpu_seeds: it refuses when seed_pre does not match the reads
    if (bad) c->seed_pre.clear();
    else c->seed_pre = pre;
    if (keep_on_device) {   // the seeds stay in HBM for pr_iter_upload_gpu_seeds
        HIPCHK(hipStreamSynchronize(s));
        if (status) std::memcpy(status, st.data(), (size_t)n_sr * 4);
        if (bad)
            return set_error(PR_ERR_CAPACITY, "%lld reads outgrew the seeding scratch (status flags, or: 0x%x)",
                             (long long)bad, bad_flags);
        return 0;
    }
    out->t = (pr_seed_task *)std::malloc(sizeof(pr_seed_task) * (size_t)(total > 0 ? total : 1));
    if (!out->t) return set_error(PR_ERR_ARG, "out of host memory");
    if (total && (rc = download(out->t, D[SB_DENSE], (size_t)total, s))) return rc;
    HIPCHK(hipStreamSynchronize(s));
    out->n = total;
    if (status) std::memcpy(status, st.data(), (size_t)n_sr * 4);
    if (bad)
        return set_error(PR_ERR_CAPACITY, "%lld reads outgrew the seeding scratch (status flags, or: 0x%x)", (long long)bad,
                         bad_flags);
    return 0;
}

extern "C" int pr_seed_gpu_seed_count(pr_ctx *c, int64_t *n) {
    if (!c || !n) return set_error(PR_ERR_ARG, "null arg");
    *n = c->seed_pre.empty() ? 0 : c->seed_pre.back();
    return 0;
}

extern "C" int pr_seed_gpu_pass2_reads(pr_ctx *c, int64_t *n) {
    if (!c || !n) return set_error(PR_ERR_ARG, "null arg");
    *n = c->seed_pass2;
    return 0;
}

extern "C" int pr_seed_gpu_last_ms(pr_ctx *c, double *ms) {
    if (!c || !ms) return set_error(PR_ERR_ARG, "null arg");
    *ms = c->ms_seed;
    return 0;
}

extern "C" int pr_seed_gpu_pass2_ms(pr_ctx *c, double *ms) {
    if (!c || !ms) return set_error(PR_ERR_ARG, "null arg");
    *ms = c->ms_seed_pass2;   // from pass 1's end to pass 2's (its status download included)
    return 0;
}

extern "C" int pr_seed_gpu_phase_ticks(pr_ctx *c, uint64_t *ticks4) {
    if (!c || !ticks4) return set_error(PR_ERR_ARG, "null arg");
    if (!c->sd[SB_NEXT].p) return set_error(PR_ERR_ARG, "no pr_seed_gpu_map launch yet");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(ticks4, c->sd[SB_NEXT].as<uint8_t>() + 64, 32, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int pr_seed_gpu_lane_ticks(pr_ctx *c, uint64_t *ticks6) {
    if (!c || !ticks6) return set_error(PR_ERR_ARG, "null arg");
    if (!c->sd[SB_NEXT].p) return set_error(PR_ERR_ARG, "no pr_seed_gpu_map launch yet");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(ticks6, c->sd[SB_NEXT].as<uint8_t>() + 64 + 4 * 8, 48, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int pr_seed_gpu_pass2_ticks(pr_ctx *c, uint64_t *t7) {
    if (!c || !t7) return set_error(PR_ERR_ARG, "null arg");
    if (!c->sd[SB_NEXT].p) return set_error(PR_ERR_ARG, "no pr_seed_gpu_map launch yet");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(t7, c->sd[SB_NEXT].as<uint8_t>() + 64 + 13 * 8, 56, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int pr_seed_gpu_occ_ticks(pr_ctx *c, uint64_t *ticks3) {
    if (!c || !ticks3) return set_error(PR_ERR_ARG, "null arg");
    if (!c->sd[SB_NEXT].p) return set_error(PR_ERR_ARG, "no pr_seed_gpu_map launch yet");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(ticks3, c->sd[SB_NEXT].as<uint8_t>() + 64 + 10 * 8, 24, hipMemcpyDeviceToHost));
    return 0;
}

// SW stage entry points are in sw_api.cpp (they share pr_ctx through this accessor)
SwResident &ctx_sw(pr_ctx *c) { return c->sw; }
hipStream_t ctx_stream(pr_ctx *c) { return c->stream; }
int ctx_device(pr_ctx *c) { return c->device; }
void ctx_sw_batch_changed(pr_ctx *c) { c->x_ready = c->x_pass = false; }
int ctx_ncu(pr_ctx *c) { return c->n_cu; }
hipEvent_t ctx_event(pr_ctx *c, int i) { return c->ev[i]; }
int pr_set_error(int code, const char *msg) { return set_error(code, "%s", msg); }
