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
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/prgpu.h"

int pr_set_error(int code, const char *msg);

namespace {

constexpr int KI = 12;                       // indexed k-mer length
constexpr uint32_t NK = 1u << (2 * KI);      // 4^12
constexpr uint8_t SEP = 5;                   // contig separator in the text
constexpr int KX = 28;                       // bases stored after each 12-mer hit (kext)
constexpr uint64_t KX_MASK = (1ull << (2 * KX)) - 1;

// 2-bit pack of s[0, n) (n <= KX), base i at bits 2i; stops at the first non-ACGT
inline uint64_t pack_ext(const uint8_t *s, int n) {
    uint64_t v = 0;
    int k = 0;
    for (; k < n && s[k] < 4; ++k) v |= (uint64_t)s[k] << (2 * k);
    return v | ((uint64_t)k << 56);
}

struct Index {
    // text: forward long reads, then the reverse complement of their concatenation
    // (bwa's forward-reverse layout), each contig followed by SEP
    std::vector<uint8_t> text;
    std::vector<int64_t> cstart;   // text offset of contig c (2*n_lr contigs in text order)
    std::vector<int32_t> cblk;     // contig containing text position (b << CB_SHIFT), per block
    std::vector<int64_t> lr_off;   // forward long-read offsets (n_lr + 1), l_pac = lr_off[n_lr]
    int n_lr = 0;
    int64_t l_pac = 0;
    std::vector<uint32_t> koff;    // [NK + 1] offsets into kpos
    std::vector<uint32_t> kpos;    // text positions of every valid 12-mer, grouped by k-mer, ascending
    std::vector<uint64_t> kext;    // per kpos entry: the next KX bases after the 12-mer (2 bits each,
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
int64_t occ(const Index &I, const uint8_t *q, int a, int b, std::vector<uint32_t> *pos = nullptr) {
    const int n = b - a;
    uint32_t code = 0;
    for (int x = a; x < a + (n < KI ? n : KI); ++x) code = (code << 2) | q[x];
    if (n < KI && !pos) return I.cnt[n - 1][code];
    if (n < KI) return -1;   // positions are only asked for seeds (>= the 12-mer length)
    if (pos) pos->clear();
    int64_t m = 0;
    const uint8_t *T = I.text.data();
    for (uint32_t r = I.koff[code]; r < I.koff[code + 1]; ++r) {
        const uint32_t p = I.kpos[r];
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
    void positions(int a, int b, std::vector<uint32_t> &pos) const { occ(I, q, a, b, &pos); }
};

// Per-read occurrence table (the seeding path): for every start a of the read, the
// 12-mer hits of q[a, a+12) with their exact match length ml = LCP(q[a..], T[p..])
// (>= 12).  occ(q[a, b)) for b - a >= 12 is #{hits of a: ml >= b - a}: a per-start
// table ge[a][t] = #{ml >= 12 + t} for t < HB, a scan of the start's hits beyond;
// shorter strings use the j-mer count tables.  Match lengths follow diagonals (when
// p-1 is a hit of a-1 with ml >= 13, p is a hit of a with ml - 1); a new diagonal
// compares the KX bases stored after the hit (kext, contiguous with kpos) and only
// goes on in the text after a full KX-base match.  Same counts as IndexOcc, one pass
// over the hits per read; the buffers are reused across the reads of a thread.
constexpr int HB = 20;

struct ReadOcc {
    const Index *I = nullptr;
    const uint8_t *q = nullptr;
    int len = 0;
    std::vector<int32_t> hoff;    // [len + 1]
    std::vector<uint32_t> hpos;   // hits of start a at [hoff[a], hoff[a+1]), text order
    std::vector<uint16_t> hml;    // their match lengths
    std::vector<uint64_t> qext;   // per start a: pack_ext of q[a+12, a+12+KX)
    std::vector<int32_t> ge;      // [len * HB]
    std::vector<int64_t> codes;   // 12-mer code per start, -1 with N

    void build(const Index &I_, const uint8_t *q_, int len_) {
        I = &I_;
        q = q_;
        len = len_;
        hoff.assign((size_t)len + 1, 0);
        qext.assign((size_t)len + 1, 0);
        hpos.clear();
        hml.clear();
        ge.assign((size_t)len * HB, 0);
        for (int a = 0; a + KI <= len; ++a) {
            const int n = len - a - KI;
            qext[a] = pack_ext(q + a + KI, n < KX ? n : KX);
        }
        const uint8_t *T = I->text.data();
        uint32_t code = 0;
        int run = 0;
        int32_t prev0 = 0, prev1 = 0;   // hits of start a-1
        // 12-mer code of every start (-1: contains N), then software prefetch of the
        // random koff / kpos / kext lines a few starts ahead (the loop is latency bound)
        codes.assign((size_t)len + 1, -1);
        for (int e = 0; e < len; ++e) {
            if (q[e] > 3) {
                run = 0;
                code = 0;
            } else {
                code = ((code << 2) | q[e]) & (NK - 1);
                ++run;
            }
            if (e - KI + 1 >= 0 && run >= KI) codes[e - KI + 1] = (int64_t)code;
        }
        constexpr int PF_OFF = 24, PF_POS = 12;
        for (int a = 0; a < PF_OFF && a < len; ++a)
            if (codes[a] >= 0) __builtin_prefetch(&I->koff[(size_t)codes[a]]);
        for (int e = KI - 1; e < len; ++e) {   // e = last base of the 12-mer starting at a = e - 11
            const int a = e - KI + 1;
            if (a + PF_OFF < len && codes[a + PF_OFF] >= 0) __builtin_prefetch(&I->koff[(size_t)codes[a + PF_OFF]]);
            if (a + PF_POS < len && codes[a + PF_POS] >= 0) {
                const uint32_t r0 = I->koff[(size_t)codes[a + PF_POS]];
                __builtin_prefetch(&I->kpos[r0]);
                __builtin_prefetch(&I->kext[r0]);
                __builtin_prefetch(&I->kext[r0] + 8);
            }
            run = codes[a] >= 0 ? KI : 0;
            code = codes[a] >= 0 ? (uint32_t)codes[a] : 0;
            hoff[a] = (int32_t)hpos.size();
            if (run >= KI) {
                int32_t k = prev0;
                int32_t *g = ge.data() + (size_t)a * HB;
                for (uint32_t r = I->koff[code]; r < I->koff[code + 1]; ++r) {
                    const uint32_t p = I->kpos[r];
                    while (k < prev1 && hpos[k] + 1 < p) ++k;
                    int ml;
                    if (k < prev1 && hpos[k] + 1 == p && hml[k] > KI) {
                        ml = hml[k] - 1;
                    } else {
                        const uint64_t ex = I->kext[r];
                        const uint64_t qe = qext[a];
                        const int le = (int)(ex >> 56), lq = (int)(qe >> 56);
                        const uint64_t x = (ex ^ qe) & KX_MASK;
                        int m = x ? __builtin_ctzll(x) >> 1 : KX;
                        m = m < le ? m : le;
                        m = m < lq ? m : lq;
                        ml = KI + m;
                        if (m == KX)
                            while (a + ml < len && q[a + ml] < 4 && T[p + ml] == q[a + ml]) ++ml;
                    }
                    hpos.push_back(p);
                    hml.push_back((uint16_t)(ml < 65535 ? ml : 65535));
                    ++g[ml - KI < HB - 1 ? ml - KI : HB - 1];
                }
                for (int t = HB - 2; t >= 0; --t) g[t] += g[t + 1];
            }
            prev0 = hoff[a];
            prev1 = (int32_t)hpos.size();
        }
        for (int a = len - KI + 1 < 0 ? 0 : len - KI + 1; a <= len; ++a) hoff[a] = (int32_t)hpos.size();
    }
    int64_t operator()(int a, int b) const {
        const int n = b - a;
        if (n < KI) {
            uint32_t code = 0;
            for (int x = a; x < b; ++x) code = (code << 2) | q[x];
            return I->cnt[n - 1][code];
        }
        if (n - KI < HB) return ge[(size_t)a * HB + (n - KI)];
        int64_t c = 0;
        for (int32_t k = hoff[a]; k < hoff[a + 1]; ++k) c += hml[k] >= n;
        return c;
    }
    void positions(int a, int b, std::vector<uint32_t> &pos) const {
        pos.clear();
        const int n = b - a;
        for (int32_t k = hoff[a]; k < hoff[a + 1]; ++k)
            if (hml[k] >= n) pos.push_back(hpos[k]);
    }
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

struct Seed {
    int64_t rbeg;   // forward-reverse coordinate (bwa): reverse strand >= l_pac
    int qbeg, len;
};
// A chain's seeds are a linked list in the read's seed pool (seeds are only ever
// appended), so chaining allocates nothing per chain.
struct Chain {
    int64_t pos;
    int rid;
    int32_t head, tail, n;   // first / last seed in the pool, seed count
    int w, kept, first;
};
struct SeedPool {
    std::vector<Seed> s;
    std::vector<int32_t> next;
    int32_t add(const Seed &x) {
        s.push_back(x);
        next.push_back(-1);
        return (int32_t)s.size() - 1;
    }
    void append(Chain &c, const Seed &x) {
        const int32_t k = add(x);
        next[c.tail] = k;
        c.tail = k;
        ++c.n;
    }
};

// text position -> bwa forward-reverse coordinate and contig (long read) id
inline void text_to_fr(const Index &I, uint32_t p, int64_t &fr, int &rid) {
    const int c = contig_of(I, p);
    const int64_t o = (int64_t)p - I.cstart[c];
    if (c < I.n_lr) {
        rid = c;
        fr = I.lr_off[c] + o;
    } else {
        rid = 2 * I.n_lr - 1 - c;   // reverse half holds the long reads in reverse order
        fr = I.l_pac + (I.l_pac - I.lr_off[rid + 1]) + o;
    }
}

bool test_and_merge(const pr_seed_opts &O, int64_t l_pac, SeedPool &P, Chain &c, const Seed &p, int rid) {
    const Seed &last = P.s[c.tail];
    const Seed &first = P.s[c.head];
    const int64_t qend = last.qbeg + last.len, rend = last.rbeg + last.len;
    if (rid != c.rid) return false;
    if (p.qbeg >= first.qbeg && p.qbeg + p.len <= qend && p.rbeg >= first.rbeg && p.rbeg + p.len <= rend)
        return true;   // contained seed
    if ((last.rbeg < l_pac || first.rbeg < l_pac) && p.rbeg >= l_pac) return false;   // other strand
    const int64_t x = p.qbeg - last.qbeg, y = p.rbeg - last.rbeg;
    if (y >= 0 && x - y <= O.w && y - x <= O.w && x - last.len < O.max_chain_gap && y - last.len < O.max_chain_gap) {
        P.append(c, p);
        return true;
    }
    return false;
}

int chain_weight(const SeedPool &P, const Chain &c) {
    int64_t end = 0;
    int w = 0;
    for (int32_t k = c.head; k >= 0; k = P.next[k]) {
        const Seed &s = P.s[k];
        if (s.qbeg >= end) w += s.len;
        else if (s.qbeg + s.len > end) w += (int)(s.qbeg + s.len - end);
        end = end > s.qbeg + s.len ? end : s.qbeg + s.len;
    }
    const int tmp = w;
    w = 0;
    end = 0;
    for (int32_t k = c.head; k >= 0; k = P.next[k]) {
        const Seed &s = P.s[k];
        if (s.rbeg >= end) w += s.len;
        else if (s.rbeg + s.len > end) w += (int)(s.rbeg + s.len - end);
        end = end > s.rbeg + s.len ? end : s.rbeg + s.len;
    }
    w = w < tmp ? w : tmp;
    return w < (1 << 30) ? w : (1 << 30) - 1;
}

struct ReadOut {
    std::vector<pr_seed_task> tasks;
};

inline int cal_max_gap(const pr_seed_opts &O, int qlen) {
    int l_del = (int)((double)(qlen * O.a - O.o_del) / O.e_del + 1.);
    int l_ins = (int)((double)(qlen * O.a - O.o_ins) / O.e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < O.w << 1 ? l : O.w << 1;
}

std::vector<uint32_t> &tl_pos() {
    static thread_local std::vector<uint32_t> v;
    return v;
}
std::vector<Chain> &tl_chains() {
    static thread_local std::vector<Chain> v;
    return v;
}

void map_read(const Index &I, const pr_seed_opts &O, const uint8_t *q, int len, int sid, ReadOut &out) {
    static thread_local ReadOcc R;
    static thread_local SeedPool P;
    static thread_local std::vector<Chain> cv;     // chains, creation order
    static thread_local std::vector<int32_t> ord;  // chain ids sorted by pos (mem_chain's btree order)
    R.build(I, q, len);
    // mem_collect_intv
    std::vector<Iv> mems, m1;
    for (int x = 0; x < len;) {
        if (q[x] < 4) {
            x = smem1(R, q, len, x, 1, m1);
            for (const Iv &p : m1)
                if (p.end - p.start >= O.min_seed_len) mems.push_back(p);
        } else {
            ++x;
        }
    }
    const int split_len = (int)(O.min_seed_len * O.split_factor + .499);
    const size_t n1 = mems.size();
    for (size_t k = 0; k < n1; ++k) {
        const Iv p = mems[k];
        if (p.end - p.start < split_len || p.occ > O.split_width) continue;
        smem1(R, q, len, (p.start + p.end) >> 1, p.occ + 1, m1);
        for (const Iv &r : m1)
            if (r.end - r.start >= O.min_seed_len) mems.push_back(r);
    }
    if (O.max_mem_intv > 0) {
        for (int x = 0; x < len;) {
            if (q[x] < 4) {
                Iv m;
                x = seed_strategy1(R, q, len, x, O.min_seed_len, O.max_mem_intv, m);
                if (m.occ > 0) mems.push_back(m);
            } else {
                ++x;
            }
        }
    }
    std::stable_sort(mems.begin(), mems.end(), [](const Iv &a, const Iv &b) {
        return a.start != b.start ? a.start < b.start : a.end < b.end;
    });
    // mem_chain: every occurrence is merged into the chain with the largest pos <= its
    // rbeg, else it opens a chain inserted after the chains of equal pos (btree order)
    P.s.clear();
    P.next.clear();
    cv.clear();
    ord.clear();
    std::vector<uint32_t> &pos = tl_pos();
    for (const Iv &p : mems) {
        const int slen = p.end - p.start;
        R.positions(p.start, p.end, pos);   // text-position order (12-mer lists are position-sorted)
        const int64_t np = (int64_t)pos.size();
        const int64_t step = np > O.max_occ ? np / O.max_occ : 1;
        int64_t count = 0;
        for (int64_t k = 0; k < np && count < O.max_occ; k += step, ++count) {
            Seed s;
            int rid;
            text_to_fr(I, pos[k], s.rbeg, rid);
            s.qbeg = p.start;
            s.len = slen;
            // first chain with pos > rbeg
            size_t lo = 0, hi = ord.size();
            while (lo < hi) {
                const size_t mid = (lo + hi) >> 1;
                if (cv[ord[mid]].pos <= s.rbeg) lo = mid + 1;
                else hi = mid;
            }
            if (lo > 0 && test_and_merge(O, I.l_pac, P, cv[ord[lo - 1]], s, rid)) continue;
            Chain c;
            c.pos = s.rbeg;
            c.rid = rid;
            c.head = c.tail = P.add(s);
            c.n = 1;
            c.w = c.kept = 0;
            c.first = -1;
            cv.push_back(c);
            ord.insert(ord.begin() + (ptrdiff_t)lo, (int32_t)cv.size() - 1);
        }
    }
    std::vector<Chain> &ch = tl_chains();
    ch.clear();
    for (int32_t id : ord) ch.push_back(cv[id]);
    // mem_chain_flt
    {
        size_t k = 0;
        for (size_t i = 0; i < ch.size(); ++i) {
            ch[i].w = chain_weight(P, ch[i]);
            if (ch[i].w >= O.min_chain_weight) {
                if (k != i) ch[k] = ch[i];
                ++k;
            }
        }
        ch.resize(k);
    }
    if (!ch.empty()) {
        std::stable_sort(ch.begin(), ch.end(), [](const Chain &a, const Chain &b) { return a.w > b.w; });
        auto cbeg = [&](const Chain &c) { return P.s[c.head].qbeg; };
        auto cend = [&](const Chain &c) { return P.s[c.tail].qbeg + P.s[c.tail].len; };
        std::vector<int> kept_idx{0};
        ch[0].kept = 3;
        for (size_t i = 1; i < ch.size(); ++i) {
            int large = 0;
            size_t k;
            for (k = 0; k < kept_idx.size(); ++k) {
                Chain &cj = ch[kept_idx[k]];
                const int bmax = cbeg(cj) > cbeg(ch[i]) ? cbeg(cj) : cbeg(ch[i]);
                const int emin = cend(cj) < cend(ch[i]) ? cend(cj) : cend(ch[i]);
                if (emin > bmax) {
                    const int li = cend(ch[i]) - cbeg(ch[i]), lj = cend(cj) - cbeg(cj);
                    const int minl = li < lj ? li : lj;
                    if (emin - bmax >= minl * O.mask_level && minl < O.max_chain_gap) {
                        large = 1;
                        if (cj.first < 0) cj.first = (int)i;
                        if (ch[i].w < cj.w * O.drop_ratio && cj.w - ch[i].w >= O.min_seed_len << 1) break;
                    }
                }
            }
            if (k == kept_idx.size()) {
                kept_idx.push_back((int)i);
                ch[i].kept = large ? 2 : 3;
            }
        }
        for (int j : kept_idx)
            if (ch[j].first >= 0) ch[ch[j].first].kept = 1;
    }
    // mem_chain2aln: the best seed of every kept chain, and the chain's reference window
    for (const Chain &c : ch) {
        if (c.kept == 0) continue;
        int32_t best = c.head;
        for (int32_t k = P.next[c.head]; k >= 0; k = P.next[k])
            if (P.s[k].len >= P.s[best].len) best = k;   // srt order: (score, index), last wins
        const Seed &s = P.s[best];
        const bool rev = s.rbeg >= I.l_pac;
        const int64_t L = I.lr_off[c.rid + 1] - I.lr_off[c.rid];
        // strand coordinates: forward long read, or its reverse complement
        const int64_t cs = rev ? I.l_pac + (I.l_pac - I.lr_off[c.rid + 1]) : I.lr_off[c.rid];
        int64_t r0 = INT64_MAX, r1 = INT64_MIN;
        for (int32_t k = c.head; k >= 0; k = P.next[k]) {
            const Seed &t = P.s[k];
            const int64_t b = t.rbeg - (t.qbeg + cal_max_gap(O, t.qbeg));
            const int64_t e = t.rbeg + t.len + ((len - t.qbeg - t.len) + cal_max_gap(O, len - t.qbeg - t.len));
            r0 = r0 < b ? r0 : b;
            r1 = r1 > e ? r1 : e;
        }
        r0 -= cs;
        r1 -= cs;
        pr_seed_task t;
        t.sr = sid;
        t.lr = c.rid;
        t.strand = rev ? 1 : 0;
        t.qbeg = s.qbeg;
        t.rbeg = (int32_t)(s.rbeg - cs);
        t.slen = s.len;
        t.rmax0 = (int32_t)(r0 > 0 ? r0 : 0);
        t.rmax1 = (int32_t)(r1 < L ? r1 : L);
        t.weight = c.w;
        t.nseed = c.n;
        out.tasks.push_back(t);
    }
}

}  // namespace

struct pr_seed_index {
    Index I;
};

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
}

extern "C" int pr_seed_index_build(const uint8_t *lr_seq, const int64_t *lr_off, int n_lr, pr_seed_index **out) {
    if (!out || n_lr < 0 || (n_lr && (!lr_seq || !lr_off))) return pr_set_error(PR_ERR_ARG, "null arg");
    *out = nullptr;
    for (int i = 0; i < n_lr; ++i)
        if (lr_off[i + 1] < lr_off[i]) return pr_set_error(PR_ERR_ARG, "lr_off not monotone");
    const int64_t l_pac = n_lr ? lr_off[n_lr] - lr_off[0] : 0;
    if (2 * l_pac + 2 * (int64_t)n_lr >= (int64_t)UINT32_MAX)
        return pr_set_error(PR_ERR_CAPACITY, "long-read shard too large for the 32-bit seed index");
    pr_seed_index *h = new pr_seed_index;
    Index &I = h->I;
    I.n_lr = n_lr;
    I.l_pac = l_pac;
    I.lr_off.assign(n_lr + 1, 0);
    for (int i = 0; i <= n_lr; ++i) I.lr_off[i] = lr_off[i] - lr_off[0];
    I.text.reserve(2 * l_pac + 2 * n_lr);
    for (int i = 0; i < n_lr; ++i) {
        I.cstart.push_back((int64_t)I.text.size());
        for (int64_t p = lr_off[i]; p < lr_off[i + 1]; ++p) I.text.push_back(lr_seq[p] < 4 ? lr_seq[p] : 4);
        I.text.push_back(SEP);
    }
    for (int i = n_lr - 1; i >= 0; --i) {
        I.cstart.push_back((int64_t)I.text.size());
        for (int64_t p = lr_off[i + 1] - 1; p >= lr_off[i]; --p) I.text.push_back(lr_seq[p] < 4 ? (uint8_t)(3 - lr_seq[p]) : 4);
        I.text.push_back(SEP);
    }
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
    std::vector<uint32_t> kc(NK, 0);
    auto for_kmers = [&](auto f) {
        uint32_t code = 0;
        int run = 0;
        for (int64_t p = 0; p < n; ++p) {
            if (T[p] > 3) { run = 0; code = 0; continue; }
            code = ((code << 2) | T[p]) & (NK - 1);
            if (++run >= KI) f(code, (uint32_t)(p - KI + 1));
        }
    };
    for_kmers([&](uint32_t c, uint32_t) { ++kc[c]; });
    I.koff.assign(NK + 1, 0);
    for (uint32_t k = 0; k < NK; ++k) I.koff[k + 1] = I.koff[k] + kc[k];
    I.kpos.resize(I.koff[NK]);
    I.kext.resize(I.koff[NK]);
    std::vector<uint32_t> fill(I.koff.begin(), I.koff.end() - 1);
    for_kmers([&](uint32_t c, uint32_t p) { I.kpos[fill[c]++] = p; });
    {   // bases after every hit, in kpos order (random text reads: spread over threads)
        const int64_t nk = (int64_t)I.kpos.size();
        int nt = (int)std::thread::hardware_concurrency();
        nt = nt < 1 ? 1 : (nt > 32 ? 32 : nt);
        auto work = [&](int t) {
            for (int64_t r = nk * t / nt; r < nk * (t + 1) / nt; ++r) {
                const uint32_t p = I.kpos[r];
                const int64_t n_after = n - ((int64_t)p + KI);   // the text ends with SEP: pack_ext stops there
                I.kext[r] = pack_ext(T + p + KI, n_after < KX ? (int)n_after : KX);
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
    }
    // j-mer counts for j < 12: C_j(x) = sum_c C_{j+1}(4x + c) + #(j-mers x ending a run of bases),
    // a run being a maximal stretch without N / SEP (an occurrence is either followed by another
    // base of its run, then it prefixes a (j+1)-mer occurrence, or it ends the run)
    std::vector<std::vector<uint32_t>> tail(KI);
    {
        int64_t s0 = 0;
        for (int64_t p = 0; p <= n; ++p) {
            if (p < n && T[p] <= 3) continue;
            for (int j = 1; j < KI && p - j >= s0; ++j) {   // run [s0, p)
                uint32_t code = 0;
                for (int64_t e = p - j; e < p; ++e) code = (code << 2) | T[e];
                tail[j].push_back(code);
            }
            s0 = p + 1;
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
                if (len > 0) map_read(h->I, *o, q.data(), len, i, res[i]);
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
