// Host seeding and chaining front end: the index / SMEM / chain part of
// `bwa-proovread index` + `bwa-proovread mem` (bin/proovread:1270, 1313) that
// turns short reads into the seed-extension task list of pr_sw_run.
//
// bwa-proovread is absent (empty submodule, .gitmodules:4-6), so this restates
// upstream bwa's published algorithms over an index of the long reads:
//   mem_collect_intv   SMEMs (bwt_smem1a) >= -k, re-seeding of long SMEMs
//                      with <= split_width hits (-r), LAST-like third round (-y)
//   mem_chain          occurrences (<= -c per SMEM, sampled in text order),
//                      chains grown by test_and_merge (-w, max_chain_gap)
//   mem_chain_flt      chain weight, -W minimum, -D drop ratio (mask_level .5)
//   mem_chain2aln      the chain's best seed (highest score, last on ties)
//                      becomes the task; the chain's reference window
//                      (rmax over all its seeds) is reported with it.
// Every algorithm works on occurrence counts of query substrings; bwa gets them
// from a bidirectional FM-index, this index answers them exactly from a 12-mer
// position table (+ j-mer count tables for lengths < 12 and verification for
// longer strings).  Parity with bwa-proovread is unpinned; deliberate
// differences: contigs are separated (bwa's concatenated pac lets a
// match run across a contig or strand boundary; such seeds are discarded there
// anyway, but they can shadow SMEMs), an N never matches (bwa substitutes random
// bases), a seed's occurrences are visited in text-position order (bwa: suffix-array
// order), ties in the chain weight sort are stable, seeds other than the best
// one of a chain are not extended.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include <sys/mman.h>

#include "../../include/prgpu.h"
#include "seed_core.h"
#include "seed_dev.h"

namespace seedc = prgpu::seedc;

int pr_set_error(int code, const char *msg);

namespace {

constexpr int KI = 12;                       // indexed k-mer length
constexpr uint32_t NK = 1u << (2 * KI);      // 4^12
constexpr uint8_t SEP = 5;                   // contig separator in the text
constexpr int KX = 28;                       // bases stored after each 12-mer hit (kext)
constexpr uint64_t KX_MASK = (1ull << (2 * KX)) - 1;

// 2-bit pack of s[0, n) (n <= KX), base i at bits 2i; stops at the first non-ACGT
// Allocator for the index's big tables: no value-initialisation on resize (the build
// writes every element, from many threads, so the pages are first touched in parallel
// instead of being zeroed by one thread), and transparent huge pages for big blocks.
template <class T>
struct BigAlloc {
    using value_type = T;
    static constexpr size_t kHuge = (size_t)32 << 20;
    BigAlloc() = default;
    template <class U>
    BigAlloc(const BigAlloc<U> &) {}
    T *allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes >= kHuge) {
            void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (p == MAP_FAILED) throw std::bad_alloc();
            madvise(p, bytes, MADV_HUGEPAGE);
            return static_cast<T *>(p);
        }
        return static_cast<T *>(::operator new(bytes));
    }
    void deallocate(T *p, size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes >= kHuge) munmap(p, bytes);
        else ::operator delete(p);
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        if constexpr (sizeof...(A) == 0) ::new ((void *)p) U;
        else ::new ((void *)p) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const BigAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const BigAlloc<U> &) const { return false; }
};
template <class T>
using BigVec = std::vector<T, BigAlloc<T>>;

struct Index {
    // text: forward long reads, then the reverse complement of their concatenation
    // (bwa's forward-reverse layout), each contig followed by SEP
    BigVec<uint8_t> text;
    std::vector<int64_t> cstart;   // text offset of contig c (2*n_lr contigs in text order)
    std::vector<int32_t> cblk;     // contig containing text position (b << CB_SHIFT), per block
    std::vector<int64_t> lr_off;   // forward long-read offsets (n_lr + 1), l_pac = lr_off[n_lr]
    int n_lr = 0;
    int64_t l_pac = 0;
    std::vector<uint64_t> koff;    // [NK + 1] offsets into kpos
    BigVec<uint32_t> kpos;         // text positions of every valid 12-mer, grouped by k-mer, ascending
                                   // (low 32 bits; seedc::hit_pos adds bit 32 from ksplit)
    std::vector<uint64_t> ksplit;  // [NK] the first hit of each k-mer at or beyond 2^32 (empty: text < 2^32)
    BigVec<uint64_t> kext;         // per kpos entry: the next KX bases after the 12-mer (2 bits each,
                                   // base i at bits 2i) and their count before N / SEP (bits 56..61)
    std::vector<uint32_t> cnt[KI]; // cnt[j][code] = occurrences of the (j+1)-mer `code` (j < KI-1)
};

constexpr int CB_SHIFT = 12;   // 4 KB blocks: the table stays cache resident

// contig of a text position: the block table gives the contig at the block start,
// the few contigs that start inside the block are stepped over
inline int contig_of(const Index &I, int64_t p) {
    int c = I.cblk[(size_t)(p >> CB_SHIFT)];
    const int nc = (int)I.cstart.size();
    while (c + 1 < nc && I.cstart[c + 1] <= p) ++c;
    return c;
}

// occurrence count of q[a, b) (codes 0-3 only), optionally collecting text positions
seedc::IndexView view_of(const Index &I);

int64_t occ(const Index &I, const uint8_t *q, int a, int b, std::vector<uint64_t> *pos = nullptr) {
    const int n = b - a;
    uint32_t code = 0;
    for (int x = a; x < a + (n < KI ? n : KI); ++x) code = (code << 2) | q[x];
    if (n < KI && !pos) return I.cnt[n - 1][code];
    if (n < KI) return -1;   // positions are only asked for seeds (>= the 12-mer length)
    if (pos) pos->clear();
    int64_t m = 0;
    const uint8_t *T = I.text.data();
    const seedc::IndexView V = view_of(I);
    for (uint64_t r = I.koff[code]; r < I.koff[code + 1]; ++r) {
        const uint64_t p = seedc::hit_pos(V, code, r);
        bool ok = true;
        for (int x = KI; x < n && ok; ++x) ok = T[p + x] == q[a + x];   // SEP / N never match
        if (ok) {
            ++m;
            if (pos) pos->push_back(p);
        }
    }
    return m;
}

struct Iv {
    int start, end;
    int64_t occ;
};

// Occurrence oracle over the index alone: every query verifies the 12-mer hits
// (diagnostic entry points pr_seed_index_occ / pr_seed_smem).
struct IndexOcc {
    const Index &I;
    const uint8_t *q;
    int64_t operator()(int a, int b) const { return occ(I, q, a, b); }
    void positions(int a, int b, std::vector<uint64_t> &pos) const { occ(I, q, a, b, &pos); }
};

// bwt_smem1a (max_intv = 0): SMEMs covering x with >= min_intv occurrences, sorted by start;
// returns the end of the longest forward match from x (the next x of the caller)
template <class Occ>
int smem1(const Occ &occ, const uint8_t *q, int len, int x, int64_t min_intv, std::vector<Iv> &mem) {
    mem.clear();
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    static thread_local std::vector<Iv> curr, prev;
    curr.clear();
    prev.clear();
    Iv ik{x, x + 1, occ(x, x + 1)};
    int i;
    for (i = x + 1; i < len; ++i) {
        if (q[i] < 4) {
            const int64_t o = occ(x, i + 1);
            if (o != ik.occ) {
                curr.push_back(ik);
                if (o < min_intv) break;
            }
            ik = Iv{x, i + 1, o};
        } else {
            curr.push_back(ik);
            break;
        }
    }
    if (i == len) curr.push_back(ik);
    std::reverse(curr.begin(), curr.end());   // longer matches first
    const int ret = curr[0].end;
    prev.swap(curr);
    for (i = x - 1; i >= -1; --i) {
        const int c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
        curr.clear();
        for (const Iv &p : prev) {
            const int64_t o = c >= 0 ? occ(i, p.end) : 0;
            if (c < 0 || o < min_intv) {
                if (curr.empty() && (mem.empty() || i + 1 < mem.back().start)) mem.push_back(Iv{i + 1, p.end, p.occ});
            } else if (curr.empty() || o != curr.back().occ) {
                curr.push_back(Iv{i, p.end, o});
            }
        }
        if (curr.empty()) break;
        prev.swap(curr);
    }
    std::reverse(mem.begin(), mem.end());
    return ret;
}

// bwt_seed_strategy1: the shortest match from x longer than min_len with < max_intv hits
template <class Occ>
int seed_strategy1(const Occ &occ, const uint8_t *q, int len, int x, int min_len, int64_t max_intv, Iv &m) {
    m = Iv{0, 0, 0};
    if (q[x] > 3) return x + 1;
    for (int i = x + 1; i < len; ++i) {
        if (q[i] > 3) return i + 1;
        if (i - x >= min_len) {
            const int64_t o = occ(x, i + 1);
            if (o < max_intv) {
                m = Iv{x, i + 1, o};
                return i + 1;
            }
        }
    }
    return len;
}

// Host path: the shared core (seed_core.h) over a view of this index, with scratch
// that grows when a read outgrows it (the device path flags such reads instead).
seedc::IndexView view_of(const Index &I) {
    seedc::IndexView v{};
    v.text = I.text.data();
    v.n_text = (int64_t)I.text.size();
    v.cstart = I.cstart.data();
    v.n_contig = (int32_t)I.cstart.size();
    v.cblk = I.cblk.data();
    v.lr_off = I.lr_off.data();
    v.n_lr = I.n_lr;
    v.l_pac = I.l_pac;
    v.koff = I.koff.data();
    v.kpos = I.kpos.data();
    v.ksplit = I.ksplit.empty() ? nullptr : I.ksplit.data();
    v.kext = I.kext.data();
    for (int j = 0; j < KI - 1; ++j) v.cnt[j] = I.cnt[j].data();
    return v;
}

struct HostScratch {
    std::vector<int32_t> hoff, codes;
    std::vector<uint64_t> qext;
    std::vector<uint32_t> ge, hpos;
    std::vector<uint8_t> hhi;
    std::vector<uint16_t> hml, rmax;
    std::vector<uint64_t> hfr;
    std::vector<seedc::Iv> mems, m1, curr, prev;
    std::vector<seedc::Seed> seeds;
    std::vector<int32_t> cnx, kept;
    std::vector<seedc::RangeEnt> htab;
    std::vector<seedc::RangeRec> rg;
    std::vector<seedc::Chain> cv, ch;
    std::vector<pr_seed_task> out;
    seedc::Scratch S{};
    int lmax = 0, hits = 1 << 14, iv = 256, mems_cap = 1024, seeds_cap = 4096, chains = 2048, out_cap = 512;
    bool hi = false;   // the index's text reaches beyond 2^32 (hhi carries bit 32 of the positions)

    void size(int len) {
        lmax = len > lmax ? len : lmax;
        hhi.resize(hi ? (size_t)hits : 0);
        hoff.resize((size_t)lmax + 1);
        codes.resize((size_t)lmax + 1);
        qext.resize((size_t)lmax + 1);
        ge.resize((size_t)lmax * seedc::HB + 1);
        rmax.resize(((size_t)lmax + 1) * seedc::RK);
        hpos.resize((size_t)hits);
        hml.resize((size_t)hits);
        hfr.resize((size_t)hits);
        mems.resize((size_t)mems_cap);
        m1.resize((size_t)iv);
        curr.resize((size_t)iv);
        prev.resize((size_t)iv);
        seeds.resize((size_t)seeds_cap);
        cv.resize((size_t)chains);
        ch.resize((size_t)chains);
        cnx.resize((size_t)chains);
        kept.resize((size_t)chains);
        const int32_t hs = seedc::range_table_size(chains);
        htab.resize((size_t)hs);
        rg.resize((size_t)chains);
        out.resize((size_t)out_cap);
        S = seedc::Scratch{lmax,        hoff.data(),  qext.data(), codes.data(), ge.data(),   hpos.data(),
                           hi ? hhi.data() : nullptr, hml.data(),  hits, mems.data(), mems_cap, m1.data(), curr.data(),
                           prev.data(), iv,           seeds.data(), seeds_cap,   cv.data(),
                           ch.data(),   cnx.data(),   kept.data(), htab.data(), rg.data(),
                           chains,      hs};
        S.rmax = rmax.data();
        S.hfr = hfr.data();
    }
    void grow(int err) {
        if (err & seedc::SC_OVER_HITS) hits *= 2;
        if (err & seedc::SC_OVER_IV) iv *= 2;
        if (err & seedc::SC_OVER_MEMS) mems_cap *= 2;
        if (err & seedc::SC_OVER_SEEDS) seeds_cap *= 2;
        if (err & seedc::SC_OVER_CHAINS) chains *= 2;
        if (err & seedc::SC_OVER_OUT) out_cap *= 2;
    }
};

struct ReadOut {
    std::vector<pr_seed_task> tasks;
};

void map_read(const seedc::IndexView &V, const pr_seed_opts &O, const uint8_t *q, int len, int sid, ReadOut &res) {
    static thread_local HostScratch H;
    const bool hi = V.ksplit != nullptr;
    if (len > H.lmax || H.S.hoff == nullptr || hi != H.hi) {
        H.hi = hi;
        H.size(len);
    }
    for (;;) {
        int n = 0;
        const int err = seedc::map_read(V, O, H.S, q, len, sid, H.out.data(), H.out_cap, &n);
        if (!err) {
            res.tasks.assign(H.out.begin(), H.out.begin() + n);
            return;
        }
        H.grow(err);
        H.size(len);
    }
}

}  // namespace

struct pr_seed_index {
    Index I;
};

namespace prgpu {
seedc::IndexView seed_index_view(const pr_seed_index *h) { return view_of(h->I); }
SeedIndexSizes seed_index_sizes(const pr_seed_index *h) {
    const Index &I = h->I;
    SeedIndexSizes z{};
    z.text = (int64_t)I.text.size();
    z.cstart = (int64_t)I.cstart.size();
    z.cblk = (int64_t)I.cblk.size();
    z.lr_off = (int64_t)I.lr_off.size();
    z.koff = (int64_t)I.koff.size();
    z.kpos = (int64_t)I.kpos.size();
    z.ksplit = (int64_t)I.ksplit.size();
    for (int j = 0; j < KI - 1; ++j) z.cnt[j] = (int64_t)I.cnt[j].size();
    return z;
}
}  // namespace prgpu

extern "C" void pr_seed_opts_default(pr_seed_opts *o, int finish) {
    std::memset(o, 0, sizeof *o);
    // bwa mem defaults + proovread.cfg bwa-sr (-k 12 -W 20 -w 40 -r 1 -D 0 -y 20) /
    // bwa-sr-finish (-k 17 -W 18 -w 30 -r 1.5 -D .75)
    o->min_seed_len = finish ? 17 : 12;
    o->min_chain_weight = finish ? 18 : 20;
    o->w = finish ? 30 : 40;
    o->split_factor = finish ? 1.5 : 1.0;
    o->split_width = 10;
    o->max_mem_intv = 20;
    o->max_occ = 500;
    o->drop_ratio = finish ? 0.75 : 0.0;
    o->max_chain_gap = 10000;
    o->mask_level = 0.5;
    o->a = 5;
    o->o_del = finish ? 15 : 2;
    o->e_del = finish ? 3 : 4;
    o->o_ins = finish ? 19 : 1;
    o->e_ins = 3;
    o->b = finish ? 13 : 11;
}

extern "C" int pr_seed_index_build(const uint8_t *lr_seq, const int64_t *lr_off, int n_lr, pr_seed_index **out) {
    if (!out || n_lr < 0 || (n_lr && (!lr_seq || !lr_off))) return pr_set_error(PR_ERR_ARG, "null arg");
    *out = nullptr;
    for (int i = 0; i < n_lr; ++i)
        if (lr_off[i + 1] < lr_off[i]) return pr_set_error(PR_ERR_ARG, "lr_off not monotone");
    const int64_t l_pac = n_lr ? lr_off[n_lr] - lr_off[0] : 0;
    if (2 * l_pac + 2 * (int64_t)n_lr > seedc::MAX_TEXT)
        return pr_set_error(PR_ERR_CAPACITY, "long reads beyond the index's 2^33 text positions (l_pac < 4.29 Gb)");
    if ((int64_t)n_lr >= ((int64_t)1 << seedc::FR_RID_BITS))
        return pr_set_error(PR_ERR_CAPACITY, "more than 2^24 long reads in one index");
    pr_seed_index *h = new pr_seed_index;
    Index &I = h->I;
    I.n_lr = n_lr;
    I.l_pac = l_pac;
    I.lr_off.assign(n_lr + 1, 0);
    for (int i = 0; i <= n_lr; ++i) I.lr_off[i] = lr_off[i] - lr_off[0];
    int nt = (int)std::thread::hardware_concurrency();
    nt = nt < 1 ? 1 : (nt > 16 ? 16 : nt);
    if (l_pac < (int64_t)1 << 21) nt = 1;
    auto run_threads = [&](auto body) {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(body, t);
        body(0);
        for (auto &x : th) x.join();
    };
    // text: forward read i at lr_off[i] + i; the reverse strand holds read n_lr-1-k as
    // contig n_lr+k, i.e. read i reverse-complemented at l_pac + n_lr + (l_pac - lr_off[i+1]) + (n_lr-1-i)
    const int64_t n_text = 2 * l_pac + 2 * (int64_t)n_lr;
    I.text.resize((size_t)n_text);
    I.cstart.assign(2 * (size_t)n_lr, 0);
    for (int i = 0; i < n_lr; ++i) {
        I.cstart[i] = I.lr_off[i] + i;
        I.cstart[2 * (size_t)n_lr - 1 - i] = l_pac + n_lr + (l_pac - I.lr_off[i + 1]) + (n_lr - 1 - i);
    }
    run_threads([&](int t) {
        uint8_t *X = I.text.data();
        for (int i = (int)((int64_t)n_lr * t / nt); i < (int)((int64_t)n_lr * (t + 1) / nt); ++i) {
            const uint8_t *r = lr_seq + lr_off[i];
            const int64_t len = lr_off[i + 1] - lr_off[i];
            uint8_t *f = X + I.cstart[i];
            uint8_t *b = X + I.cstart[2 * (size_t)n_lr - 1 - i];
            for (int64_t p = 0; p < len; ++p) {
                const uint8_t c = seedc::base_code(r[p]);
                f[p] = c;
                b[len - 1 - p] = c < 4 ? (uint8_t)(3 - c) : 4;
            }
            f[len] = SEP;
            b[len] = SEP;
        }
    });
    // 12-mer table (positions ascending within a k-mer)
    const uint8_t *T = I.text.data();
    const int64_t n = (int64_t)I.text.size();
    {
        const int64_t nb = (n >> CB_SHIFT) + 1;
        I.cblk.assign((size_t)nb, 0);
        int c = 0;
        const int nc = (int)I.cstart.size();
        for (int64_t b = 0; b < nb; ++b) {
            while (c + 1 < nc && I.cstart[c + 1] <= (b << CB_SHIFT)) ++c;
            I.cblk[(size_t)b] = c;
        }
    }
    // k-mers starting in [p0, p1) (a k-mer may read past p1)
    auto for_kmers = [&](int64_t p0, int64_t p1, auto f) {
        uint32_t code = 0;
        int run = 0;
        int64_t p = p0 - (KI - 1) > 0 ? p0 - (KI - 1) : 0;
        for (; p < p1 + KI - 1 && p < n; ++p) {
            if (T[p] > 3) { run = 0; code = 0; continue; }
            code = ((code << 2) | T[p]) & (NK - 1);
            if (++run >= KI && p - KI + 1 >= p0) f(code, (int64_t)(p - KI + 1));
        }
    };
    // counting split over text chunks (per-chunk counts, each thread zeroing and filling
    // its own table), then the table offsets summed over k-mer ranges in parallel
    std::vector<std::vector<uint32_t>> tc((size_t)nt);
    run_threads([&](int t) {
        std::vector<uint32_t> &c = tc[(size_t)t];
        c.assign(NK, 0);
        for_kmers(n * t / nt, n * (t + 1) / nt, [&](uint32_t k, int64_t) { ++c[k]; });
    });
    std::vector<uint32_t> kc(NK);
    I.koff.assign(NK + 1, 0);
    std::vector<uint64_t> part((size_t)nt + 1, 0);
    run_threads([&](int t) {
        const uint32_t k0 = (uint32_t)((uint64_t)NK * t / nt), k1 = (uint32_t)((uint64_t)NK * (t + 1) / nt);
        uint64_t run = 0;
        for (uint32_t k = k0; k < k1; ++k) {
            uint32_t sum = 0;
            for (int u = 0; u < nt; ++u) sum += tc[(size_t)u][k];
            kc[k] = sum;
            run += sum;
            I.koff[k + 1] = run;   // range-local prefix, shifted below
        }
        part[(size_t)t + 1] = run;
    });
    for (int t = 0; t < nt; ++t) part[(size_t)t + 1] += part[(size_t)t];
    run_threads([&](int t) {
        const uint32_t k0 = (uint32_t)((uint64_t)NK * t / nt), k1 = (uint32_t)((uint64_t)NK * (t + 1) / nt);
        const uint64_t base = part[(size_t)t];
        for (uint32_t k = k0; k < k1; ++k) I.koff[k + 1] += base;
    });
    I.kpos.resize(I.koff[NK]);
    I.kext.resize(I.koff[NK]);
    // Fill in two cache-friendly passes instead of one scatter over the whole table:
    //  1. every thread walks its text chunk once, computing the k-mer code and the KX bases
    //     after it with rolling windows (sequential reads), and appends (pos, low k-mer bits,
    //     ext) to one of NB buckets by the high k-mer bits (NB sequential write streams);
    //  2. every bucket (a contiguous koff range, ~1/NB of the table) is counting-sorted by
    //     the low bits into kpos / kext, writes staying inside the bucket's region.
    // A bucket holds thread 0's records, then thread 1's ..., each in text order, and pass 2
    // is stable, so every k-mer's positions stay in ascending text order.
    constexpr int LB = 12;                    // low k-mer bits sorted in pass 2
    constexpr uint32_t NB = NK >> LB;         // buckets
    struct Rec {
        uint32_t pos, low;   // low 32 bits of the position; the k-mer's low bits | bit 32 of the position << 31
        uint64_t ext;
    };
    const bool paged = n > (int64_t)seedc::POS_PAGE;
    if (paged) I.ksplit.assign(NK, 0);
    BigVec<Rec> tmp(I.koff[NK]);
    {
        // per-thread bucket cursors: bucket b starts at koff[b << LB]; thread t after threads < t
        std::vector<std::vector<uint64_t>> cur((size_t)nt, std::vector<uint64_t>(NB, 0));
        run_threads([&](int u) {
            for (uint32_t b = (uint32_t)((uint64_t)NB * u / nt); b < (uint32_t)((uint64_t)NB * (u + 1) / nt); ++b) {
                uint64_t o = I.koff[b << LB];
                for (int t = 0; t < nt; ++t) {
                    cur[(size_t)t][b] = o;
                    uint64_t sz = 0;
                    for (uint32_t k = b << LB; k < ((b + 1) << LB); ++k) sz += tc[(size_t)t][k];
                    o += sz;
                }
            }
        });
        tc.clear();
        tc.shrink_to_fit();
        run_threads([&](int t) {
            const int64_t p0 = n * t / nt, p1 = n * (t + 1) / nt;
            uint64_t *c = cur[(size_t)t].data();
            Rec *R = tmp.data();
            uint32_t code = 0;
            int run = 0;
            int64_t p = p0 - (KI - 1) > 0 ? p0 - (KI - 1) : 0;
            // w: bases T[p+1 .. p+1+KX) two bits each (non-bases as 0); nb: first index >= p+1
            // holding N / SEP (the text ends with SEP, so nb < n always exists)
            uint64_t w = 0;
            for (int j = KX - 1; j >= 0; --j) w = (w << 2) | (p + 1 + j < n ? (uint64_t)(T[p + 1 + j] & 3) : 0);
            int64_t nb = p + 1;
            while (nb < n && T[nb] <= 3) ++nb;
            for (bool first = true; p < p1 + KI - 1 && p < n; ++p, first = false) {
                if (!first) {   // slide the windows from p-1 to p
                    const int64_t q = p + KX;
                    w = (w >> 2) | ((q < n ? (uint64_t)(T[q] & 3) : 0) << (2 * (KX - 1)));
                    if (nb < p + 1) {
                        nb = p + 1;
                        while (nb < n && T[nb] <= 3) ++nb;
                    }
                }
                if (T[p] > 3) { run = 0; code = 0; continue; }
                code = ((code << 2) | T[p]) & (NK - 1);
                if (++run >= KI && p - KI + 1 >= p0) {
                    int64_t m = nb - (p + 1);
                    if (m > KX) m = KX;
                    const uint64_t ext = (m ? (w & ((1ull << (2 * m)) - 1)) : 0) | ((uint64_t)m << 56);
                    Rec &r = R[c[code >> LB]++];
                    r.pos = (uint32_t)(p - KI + 1);
                    r.low = (code & ((1u << LB) - 1)) | ((uint32_t)((uint64_t)(p - KI + 1) >> 32) << 31);
                    r.ext = ext;
                }
            }
        });
    }
    {
        std::atomic<uint32_t> next{0};
        run_threads([&](int) {
            std::vector<uint64_t> fill((size_t)1 << LB);
            for (uint32_t b; (b = next.fetch_add(1)) < NB;) {
                const uint32_t k0 = b << LB;
                for (uint32_t j = 0; j < (1u << LB); ++j) fill[j] = I.koff[k0 + j];
                if (paged)   // no hit beyond 2^32 yet: the split is the list's end
                    for (uint32_t j = 0; j < (1u << LB); ++j) I.ksplit[k0 + j] = I.koff[k0 + j + 1];
                for (uint64_t i = I.koff[k0]; i < I.koff[k0 + (1u << LB)]; ++i) {
                    const Rec &r = tmp[i];
                    const uint32_t lo = r.low & ((1u << LB) - 1);
                    const uint64_t slot = fill[lo]++;
                    if ((r.low >> 31) && I.ksplit[k0 + lo] > slot) I.ksplit[k0 + lo] = slot;   // text order
                    I.kpos[slot] = r.pos;
                    I.kext[slot] = r.ext;
                }
            }
        });
    }
    tmp.clear();
    tmp.shrink_to_fit();
    // j-mer counts for j < 12: C_j(x) = sum_c C_{j+1}(4x + c) + #(j-mers x ending a run of bases),
    // a run being a maximal stretch without N / SEP (an occurrence is either followed by another
    // base of its run, then it prefixes a (j+1)-mer occurrence, or it ends the run)
    std::vector<std::vector<uint32_t>> tail(KI);
    {
        // the positions that end a run of bases (a non-base after a base; the text ends with
        // SEP), one list per text chunk; the j-mers (j < 12) ending just before each
        std::vector<std::vector<int64_t>> stops((size_t)nt);
        run_threads([&](int t) {
            for (int64_t p = n * t / nt; p < n * (t + 1) / nt; ++p)
                if (T[p] > 3 && p > 0 && T[p - 1] <= 3) stops[(size_t)t].push_back(p);
        });
        for (auto &v : stops)
            for (const int64_t p : v) {
                uint32_t code = 0;
                for (int j = 1; j < KI && p - j >= 0 && T[p - j] <= 3; ++j) {
                    code |= (uint32_t)T[p - j] << (2 * (j - 1));   // T[p-j] starts the j-mer
                    tail[j].push_back(code);
                }
            }
    }
    I.cnt[KI - 1] = std::move(kc);
    for (int j = KI - 1; j >= 1; --j) {
        std::vector<uint32_t> &cj = I.cnt[j - 1];
        cj.assign((size_t)1 << (2 * j), 0);
        const std::vector<uint32_t> &cn = I.cnt[j];
        for (size_t x = 0; x < cj.size(); ++x) cj[x] = cn[4 * x] + cn[4 * x + 1] + cn[4 * x + 2] + cn[4 * x + 3];
        for (uint32_t code : tail[j]) ++cj[code];
    }
    *out = h;
    return 0;
}

extern "C" void pr_seed_index_free(pr_seed_index *h) { delete h; }

// order-sensitive 64-bit digests of the index tables (test hook: a faster build must
// produce identical tables)
template <class T>
static uint64_t digest_of(const T *p, size_t n) {
    uint64_t h = 1469598103934665603ull ^ (uint64_t)n;
    for (size_t i = 0; i < n; ++i) {
        h ^= (uint64_t)p[i];
        h *= 1099511628211ull;
        h ^= h >> 29;
    }
    return h;
}

template <class A, class B, class Cc, class Dd, class E, class F, class G, class H>
static void digest6(const A &text, const B &koff, const Cc &kpos, const Dd &kext, const E &cnt, const F &cstart,
                    const G &cblk, const H &lr_off, uint64_t *out6) {
    out6[0] = digest_of(text.data(), text.size());
    out6[1] = digest_of(koff.data(), koff.size());
    out6[2] = digest_of(kpos.data(), kpos.size());
    out6[3] = digest_of(kext.data(), kext.size());
    uint64_t c = 0;
    for (int j = 0; j < KI; ++j) c = c * 31 + digest_of(cnt[j].data(), cnt[j].size());
    out6[4] = c;
    out6[5] = digest_of(cstart.data(), cstart.size()) * 31 + digest_of(cblk.data(), cblk.size()) * 7 +
              digest_of(lr_off.data(), lr_off.size());
}

extern "C" int pr_seed_index_digest(const pr_seed_index *h, uint64_t *out6) {
    if (!h || !out6) return pr_set_error(PR_ERR_ARG, "null arg");
    const Index &I = h->I;
    digest6(I.text, I.koff, I.kpos, I.kext, I.cnt, I.cstart, I.cblk, I.lr_off, out6);
    if (!I.ksplit.empty()) out6[1] ^= digest_of(I.ksplit.data(), I.ksplit.size()) * 31;   // texts beyond 2^32
    return 0;
}

// test hook: the k-mer offsets [NK + 1] and (texts beyond 2^32) the page splits [NK]
extern "C" int pr_seed_index_koff(const pr_seed_index *h, uint64_t *koff, uint64_t *ksplit) {
    if (!h || !koff) return pr_set_error(PR_ERR_ARG, "null arg");
    std::memcpy(koff, h->I.koff.data(), h->I.koff.size() * 8);
    if (ksplit && !h->I.ksplit.empty()) std::memcpy(ksplit, h->I.ksplit.data(), h->I.ksplit.size() * 8);
    return 0;
}

namespace prgpu {
void seed_digest_tables(const std::vector<uint8_t> &text, const std::vector<uint64_t> &koff,
                        const std::vector<uint32_t> &kpos, const std::vector<uint64_t> &kext,
                        const std::vector<std::vector<uint32_t>> &cnt, const std::vector<int64_t> &cstart,
                        const std::vector<int32_t> &cblk, const std::vector<int64_t> &lr_off,
                        const std::vector<uint64_t> &ksplit, uint64_t *out6) {
    digest6(text, koff, kpos, kext, cnt, cstart, cblk, lr_off, out6);
    if (!ksplit.empty()) out6[1] ^= digest_of(ksplit.data(), ksplit.size()) * 31;
}
}  // namespace prgpu

extern "C" int pr_seed_index_occ(const pr_seed_index *h, const uint8_t *s, int n, int64_t *count) {
    if (!h || !s || !count || n <= 0) return pr_set_error(PR_ERR_ARG, "bad arg");
    for (int i = 0; i < n; ++i)
        if (s[i] > 3) { *count = 0; return 0; }
    *count = occ(h->I, s, 0, n);
    return 0;
}

extern "C" int pr_seed_smem(const pr_seed_index *h, const uint8_t *q, int len, int x, int64_t min_intv,
                            int32_t *start, int32_t *end, int64_t *occs, int cap, int *n_out) {
    if (!h || !q || !n_out || x < 0 || x >= len) return pr_set_error(PR_ERR_ARG, "bad arg");
    std::vector<Iv> mem;
    const int ret = smem1(IndexOcc{h->I, q}, q, len, x, min_intv, mem);
    if ((int)mem.size() > cap) return pr_set_error(PR_ERR_CAPACITY, "smem output capacity");
    for (size_t i = 0; i < mem.size(); ++i) start[i] = mem[i].start, end[i] = mem[i].end, occs[i] = mem[i].occ;
    *n_out = (int)mem.size();
    return ret;
}

extern "C" int pr_seed_map(const pr_seed_index *h, const pr_seed_opts *o, const uint8_t *sr_seq, const int64_t *sr_off,
                           int n_sr, int n_threads, pr_seed_tasks *out) {
    if (!h || !o || !out || n_sr < 0 || (n_sr && (!sr_seq || !sr_off))) return pr_set_error(PR_ERR_ARG, "null arg");
    if (o->min_seed_len < KI) return pr_set_error(PR_ERR_UNSUPPORTED, "min seed length below the 12-mer index");
    if (o->max_occ <= 0 || o->w < 0) return pr_set_error(PR_ERR_ARG, "bad seeding options");
    out->n = 0;
    out->t = nullptr;
    for (int i = 0; i < n_sr; ++i)
        if (sr_off[i + 1] < sr_off[i] || sr_off[i + 1] - sr_off[i] > (1 << 20))
            return pr_set_error(PR_ERR_ARG, "sr_off not monotone");
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = nt < 1 ? 1 : (nt > 256 ? 256 : nt);
    std::vector<ReadOut> res(n_sr);
    const seedc::IndexView V = view_of(h->I);
    std::atomic<int> next{0};
    auto work = [&]() {
        std::vector<uint8_t> q;
        for (;;) {
            const int i0 = next.fetch_add(64);
            if (i0 >= n_sr) break;
            for (int i = i0; i < n_sr && i < i0 + 64; ++i) {
                const int len = (int)(sr_off[i + 1] - sr_off[i]);
                q.assign(sr_seq + sr_off[i], sr_seq + sr_off[i + 1]);
                for (auto &c : q) c = c < 4 ? c : 4;
                if (len > 0) map_read(V, *o, q.data(), len, i, res[i]);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    int64_t total = 0;
    for (auto &r : res) total += (int64_t)r.tasks.size();
    out->t = (pr_seed_task *)std::malloc(sizeof(pr_seed_task) * (size_t)(total > 0 ? total : 1));
    if (!out->t) return pr_set_error(PR_ERR_ARG, "out of host memory");
    int64_t k = 0;
    for (auto &r : res)
        for (auto &t : r.tasks) out->t[k++] = t;
    out->n = total;
    return 0;
}

extern "C" void pr_seed_tasks_free(pr_seed_tasks *t) {
    if (t && t->t) std::free(t->t);
    if (t) t->t = nullptr, t->n = 0;
}

// The device path's arithmetic on the host: seed_core.h with the device's fixed
// scratch capacities (seedc::device_caps), so tests can check which reads the GPU
// kernel flags and that every other read gets the host path's tasks.
extern "C" int pr_seed_map_device_caps(const pr_seed_index *h, const pr_seed_opts *o, const uint8_t *sr_seq,
                                       const int64_t *sr_off, int n_sr, int n_threads, pr_seed_tasks *out,
                                       int32_t *status) {
    if (!h || !o || !out || !status || n_sr < 0 || (n_sr && (!sr_seq || !sr_off)))
        return pr_set_error(PR_ERR_ARG, "null arg");
    if (o->min_seed_len < KI) return pr_set_error(PR_ERR_UNSUPPORTED, "min seed length below the 12-mer index");
    out->n = 0;
    out->t = nullptr;
    seedc::IndexView V = view_of(h->I);
    int qmax = 1;
    for (int i = 0; i < n_sr; ++i) qmax = std::max<int>(qmax, (int)(sr_off[i + 1] - sr_off[i]));
    // the device's 4-bit text (16 bases a word, SEP past the end, 8 padding words), so the lazy
    // table's 64-base text walks run here as on the device
    std::vector<uint64_t> text4((size_t)(V.n_text / 16 + 8), 0);
    for (size_t w = 0; w < text4.size(); ++w) {
        uint64_t v = 0;
        for (int k = 0; k < 16; ++k) {
            const int64_t x = (int64_t)w * 16 + k;
            v |= (uint64_t)(x < V.n_text ? V.text[x] : SEP) << (4 * k);
        }
        text4[w] = v;
    }
    V.text4 = text4.data();
    seedc::Caps caps = seedc::device_caps(qmax);   // (the output slots follow the longest read, as on the device)
    caps.hi = V.ksplit != nullptr;
    caps.lazy = seedc::lazy_occ(*o) ? 1 : 0;   // the device's pass-1 table for these options
    const int64_t bytes = seedc::scratch_bytes(caps);
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = nt < 1 ? 1 : (nt > 64 ? 64 : nt);
    std::vector<ReadOut> res(n_sr);
    std::atomic<int> next{0};
    // PRGPU_SCRATCH_FILL=<byte>: the slabs start filled with that byte instead of zeros -- device
    // scratch is never cleared, so a result that depends on the fill is a read of stale scratch
    const char *fe = getenv("PRGPU_SCRATCH_FILL");
    const uint64_t fill = fe ? 0x0101010101010101ull * (uint64_t)(strtoul(fe, nullptr, 0) & 0xFF) : 0;
    auto work = [&]() {
        std::vector<uint64_t> slab((size_t)(bytes / 8 + 1), fill);
        seedc::Scratch S = seedc::carve(reinterpret_cast<uint8_t *>(slab.data()), caps);
        std::vector<pr_seed_task> buf((size_t)caps.out);
        std::vector<uint64_t> big;
        for (;;) {
            const int i = next.fetch_add(1);
            if (i >= n_sr) break;
            const int len = (int)(sr_off[i + 1] - sr_off[i]);
            int n = 0, err = 0;
            if (len > 0) err = seedc::map_read(V, *o, S, sr_seq + sr_off[i], len, i, buf.data(), caps.out, &n);
            // the device's later passes: the arrays that overflowed grown, up to 4 times
            seedc::Caps cg = caps;
            for (int pass = 3; pass <= 6 && err && !(err & (seedc::SC_OVER_LEN | seedc::SC_OVER_OUT)); ++pass) {
                if (err & seedc::SC_OVER_HITS) cg.hits *= 4;
                if (err & seedc::SC_OVER_IV) cg.iv *= 2;
                if (err & seedc::SC_OVER_MEMS) cg.mems *= 2;
                if (err & seedc::SC_OVER_SEEDS) cg.seeds *= 2;
                if (err & seedc::SC_OVER_CHAINS) cg.chains *= 2;
                big.assign((size_t)(seedc::scratch_bytes(cg) / 8 + 1), fill);
                seedc::Scratch G = seedc::carve(reinterpret_cast<uint8_t *>(big.data()), cg);
                err = seedc::map_read(V, *o, G, sr_seq + sr_off[i], len, i, buf.data(), caps.out, &n);
            }
            status[i] = err;
            if (!err) res[i].tasks.assign(buf.begin(), buf.begin() + n);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    int64_t total = 0;
    for (auto &r : res) total += (int64_t)r.tasks.size();
    out->t = (pr_seed_task *)std::malloc(sizeof(pr_seed_task) * (size_t)(total > 0 ? total : 1));
    if (!out->t) return pr_set_error(PR_ERR_ARG, "out of host memory");
    int64_t k = 0;
    for (auto &r : res)
        for (auto &t : r.tasks) out->t[k++] = t;
    out->n = total;
    return 0;
}
