// SAM text -> BAM records and BGZF compression for the samtools drop-in (SURVEY.md
// §8f.3: `samtools view -bS` after bwa-proovread, bin/proovread:1313).  Host code,
// threads over line ranges / BGZF blocks.  Byte-identical to proovread_amd/bamio.py
// (sam_to_record, BgzfWriter): same record layout (SAM/BAM spec), smallest-fitting
// integer tag type in the order c, C, s, S, i, I, and the same zlib raw-deflate
// parameters per 0xFF00-byte block.
#include <charconv>
#include <cmath>
#include <cstdio>
#include <stdint.h>
#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/prgpu.h"

int pr_set_error(int code, const char *msg);

namespace {

const char OPS[] = "MIDNSHP=X";

int nt16(char c) {
    switch (c >= 'a' && c <= 'z' ? c - 32 : c) {
        case '=': return 0;
        case 'A': return 1;
        case 'C': return 2;
        case 'M': return 3;
        case 'G': return 4;
        case 'R': return 5;
        case 'S': return 6;
        case 'V': return 7;
        case 'T': return 8;
        case 'W': return 9;
        case 'Y': return 10;
        case 'H': return 11;
        case 'K': return 12;
        case 'D': return 13;
        case 'B': return 14;
        default: return 15;
    }
}

int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

template <class T>
void put(std::string &o, T v) {
    o.append(reinterpret_cast<const char *>(&v), sizeof v);
}

bool parse_i64(const char *s, const char *e, int64_t &v) {
    std::string t(s, e);
    char *end = nullptr;
    v = std::strtoll(t.c_str(), &end, 10);
    return end && *end == 0 && !t.empty();
}

// One SAM line [s, e) -> record (block_size prefix included) appended to o; false if malformed.
bool encode_line(const char *s, const char *e, const std::unordered_map<std::string, int> &ref, std::string &o) {
    std::vector<std::pair<const char *, const char *>> f;
    const char *p = s;
    for (const char *q = s; q <= e; ++q)
        if (q == e || *q == '\t') {
            f.emplace_back(p, q);
            p = q + 1;
        }
    if (f.size() < 11) return false;
    auto str = [&](int i) { return std::string(f[i].first, f[i].second); };
    int64_t flag, pos, mapq, pnext, tlen;
    if (!parse_i64(f[1].first, f[1].second, flag) || !parse_i64(f[3].first, f[3].second, pos) ||
        !parse_i64(f[4].first, f[4].second, mapq) || !parse_i64(f[7].first, f[7].second, pnext) ||
        !parse_i64(f[8].first, f[8].second, tlen))
        return false;
    // CIGAR
    std::vector<uint32_t> ops;
    const std::string cig = str(5);
    if (cig != "*") {
        int64_t num = 0;
        bool have = false;
        for (char c : cig) {
            if (c >= '0' && c <= '9') {
                num = num * 10 + (c - '0');
                have = true;
            } else {
                const char *k = std::strchr(OPS, c);
                if (!k || !*k || !have) return false;
                ops.push_back((uint32_t)(num << 4) | (uint32_t)(k - OPS));
                num = 0;
                have = false;
            }
        }
    }
    int64_t span = 0;
    for (uint32_t x : ops) {
        const int op = x & 15;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) span += x >> 4;
    }
    const std::string rname = str(2), rnext = str(6), qname = str(0);
    auto rid_of = [&](const std::string &n) {
        auto it = ref.find(n);
        return it == ref.end() ? -1 : it->second;
    };
    const int32_t rid = rname != "*" ? rid_of(rname) : -1;
    const int32_t nid = rnext == "=" ? rid : (rnext != "*" ? rid_of(rnext) : -1);
    const int64_t beg = pos - 1;
    const int64_t end = beg + (span ? span : 1);
    const std::string seq = str(9), qual = str(10);
    const int32_t l_seq = seq == "*" ? 0 : (int32_t)seq.size();
    std::string body;
    put<int32_t>(body, rid);
    put<int32_t>(body, (int32_t)beg);
    put<uint8_t>(body, (uint8_t)(qname.size() + 1));
    put<uint8_t>(body, (uint8_t)mapq);
    put<uint16_t>(body, (uint16_t)(beg >= 0 ? reg2bin(beg, end) : 4680));
    put<uint16_t>(body, (uint16_t)ops.size());
    put<uint16_t>(body, (uint16_t)flag);
    put<int32_t>(body, l_seq);
    put<int32_t>(body, nid);
    put<int32_t>(body, (int32_t)(pnext - 1));
    put<int32_t>(body, (int32_t)tlen);
    body += qname;
    body.push_back('\0');
    for (uint32_t x : ops) put<uint32_t>(body, x);
    std::string sb((size_t)(l_seq + 1) / 2, '\0');
    for (int32_t i = 0; i < l_seq; ++i) sb[(size_t)i >> 1] = (char)(sb[(size_t)i >> 1] | (nt16(seq[i]) << (4 * (1 - (i & 1)))));
    body += sb;
    if (qual == "*") {
        body.append((size_t)l_seq, (char)0xFF);
    } else {
        const size_t nq = std::min(qual.size(), (size_t)l_seq);
        for (size_t i = 0; i < nq; ++i) body.push_back((char)(qual[i] - 33));
    }
    // optional fields
    for (size_t k = 11; k < f.size(); ++k) {
        const std::string t = str((int)k);
        if (t.size() < 5 || t[2] != ':' || t[4] != ':') return false;
        const std::string tag = t.substr(0, 2), val = t.substr(5);
        const char typ = t[3];
        if (typ == 'i') {
            int64_t v;
            if (!parse_i64(val.data(), val.data() + val.size(), v)) return false;
            body += tag;
            if (v >= -128 && v <= 127) { body.push_back('c'); put<int8_t>(body, (int8_t)v); }
            else if (v >= 0 && v <= 255) { body.push_back('C'); put<uint8_t>(body, (uint8_t)v); }
            else if (v >= -32768 && v <= 32767) { body.push_back('s'); put<int16_t>(body, (int16_t)v); }
            else if (v >= 0 && v <= 65535) { body.push_back('S'); put<uint16_t>(body, (uint16_t)v); }
            else if (v >= INT32_MIN && v <= INT32_MAX) { body.push_back('i'); put<int32_t>(body, (int32_t)v); }
            else if (v >= 0 && v <= (int64_t)UINT32_MAX) { body.push_back('I'); put<uint32_t>(body, (uint32_t)v); }
            else return false;
        } else if (typ == 'f') {
            body += tag;
            body.push_back('f');
            put<float>(body, (float)std::strtod(val.c_str(), nullptr));
        } else if (typ == 'A') {
            body += tag;
            body.push_back('A');
            if (!val.empty()) body.push_back(val[0]);
        } else if (typ == 'B') {
            if (val.empty()) return false;
            const char st = val[0];
            std::vector<std::string> xs;
            size_t a = 2;
            while (a <= val.size() && val.size() > 1) {
                size_t b = val.find(',', a);
                if (b == std::string::npos) b = val.size();
                xs.push_back(val.substr(a, b - a));
                a = b + 1;
            }
            body += tag;
            body.push_back('B');
            body.push_back(st);
            put<int32_t>(body, (int32_t)xs.size());
            for (const std::string &x : xs) {
                if (st == 'f') { put<float>(body, (float)std::strtod(x.c_str(), nullptr)); continue; }
                int64_t v;
                if (!parse_i64(x.data(), x.data() + x.size(), v)) return false;
                switch (st) {
                    case 'c': put<int8_t>(body, (int8_t)v); break;
                    case 'C': put<uint8_t>(body, (uint8_t)v); break;
                    case 's': put<int16_t>(body, (int16_t)v); break;
                    case 'S': put<uint16_t>(body, (uint16_t)v); break;
                    case 'i': put<int32_t>(body, (int32_t)v); break;
                    case 'I': put<uint32_t>(body, (uint32_t)v); break;
                    default: return false;
                }
            }
        } else {   // Z, H
            body += tag;
            body.push_back(typ);
            body += val;
            body.push_back('\0');
        }
    }
    put<int32_t>(o, (int32_t)body.size());
    o += body;
    return true;
}

uint8_t *take(const std::string &s, int64_t *len) {
    uint8_t *p = (uint8_t *)std::malloc(s.size() ? s.size() : 1);
    if (p && !s.empty()) std::memcpy(p, s.data(), s.size());
    *len = (int64_t)s.size();
    return p;
}

}  // namespace

extern "C" int pr_sam_encode(const char *text, int64_t len, const char *const *ref_names, int32_t n_ref, int n_threads,
                             uint8_t **out, int64_t *out_len, int64_t *n_records) {
    if (!out || !out_len || (len && !text) || n_ref < 0 || (n_ref && !ref_names)) return pr_set_error(PR_ERR_ARG, "null arg");
    std::unordered_map<std::string, int> ref;
    for (int i = 0; i < n_ref; ++i) ref[ref_names[i]] = i;   // a repeated name maps to its last entry, like the dict
    // line starts (header lines '@' and empty lines skipped)
    std::vector<std::pair<int64_t, int64_t>> lines;
    for (int64_t i = 0; i < len;) {
        int64_t j = i;
        while (j < len && text[j] != '\n') ++j;
        int64_t e = j;
        if (e > i && text[e - 1] == '\r') --e;
        if (e > i && text[i] != '@') lines.emplace_back(i, e);
        i = j + 1;
    }
    const int64_t n = (int64_t)lines.size();
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    if (n < 4096) nt = 1;
    std::vector<std::string> part((size_t)nt);
    std::vector<int64_t> bad((size_t)nt, -1);
    auto work = [&](int t) {
        for (int64_t k = n * t / nt; k < n * (t + 1) / nt; ++k)
            if (!encode_line(text + lines[k].first, text + lines[k].second, ref, part[t])) {
                bad[t] = k;
                return;
            }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    for (int t = 0; t < nt; ++t)
        if (bad[t] >= 0) return pr_set_error(PR_ERR_SAM, "malformed SAM record");
    std::string all;
    size_t tot = 0;
    for (auto &p : part) tot += p.size();
    all.reserve(tot);
    for (auto &p : part) all += p;
    *out = take(all, out_len);
    if (n_records) *n_records = n;
    return *out ? 0 : pr_set_error(PR_ERR_ARG, "out of host memory");
}

extern "C" int pr_bgzf_compress(const uint8_t *data, int64_t len, int level, int n_threads, uint8_t **out,
                                int64_t *out_len) {
    if (!out || !out_len || (len && !data)) return pr_set_error(PR_ERR_ARG, "null arg");
    const int64_t BS = 0xFF00;
    const int64_t nb = (len + BS - 1) / BS;
    std::vector<std::string> blk((size_t)nb);
    std::vector<int> fail((size_t)(nb ? nb : 1), 0);
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    if (nb < 2) nt = 1;
    auto work = [&](int t) {
        std::vector<uint8_t> buf(compressBound(BS) + 64);
        for (int64_t b = t; b < nb; b += nt) {
            const uint8_t *src = data + b * BS;
            const uInt n = (uInt)std::min(BS, len - b * BS);
            z_stream z;
            std::memset(&z, 0, sizeof z);
            if (deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) { fail[b] = 1; continue; }
            z.next_in = const_cast<Bytef *>(src);
            z.avail_in = n;
            z.next_out = buf.data();
            z.avail_out = (uInt)buf.size();
            const int rc = deflate(&z, Z_FINISH);
            const size_t clen = buf.size() - z.avail_out;
            deflateEnd(&z);
            if (rc != Z_STREAM_END || clen + 25 > 65536) { fail[b] = 1; continue; }
            std::string &o = blk[(size_t)b];
            const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0,
                                     (uint8_t)((clen + 25) & 0xFF), (uint8_t)((clen + 25) >> 8)};
            o.append(reinterpret_cast<const char *>(hdr), 18);
            o.append(reinterpret_cast<const char *>(buf.data()), clen);
            const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), src, n);
            put<uint32_t>(o, crc);
            put<uint32_t>(o, (uint32_t)n);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    for (int64_t b = 0; b < nb; ++b)
        if (fail[b]) return pr_set_error(PR_ERR_ARG, "deflate failed");
    std::string all;
    for (auto &b : blk) all += b;
    *out = take(all, out_len);
    return *out ? 0 : pr_set_error(PR_ERR_ARG, "out of host memory");
}

// BGZF bytes -> the uncompressed stream.  Block boundaries are found by one serial walk
// over the BC extra fields (BSIZE) and each block's ISIZE trailer, then the blocks are
// inflated in parallel straight into their place in the output (samtools sort's input side,
// bin/proovread:1338).
extern "C" int pr_bgzf_decompress(const uint8_t *data, int64_t len, int n_threads, uint8_t **out, int64_t *out_len) {
    if (!out || !out_len || (len && !data)) return pr_set_error(PR_ERR_ARG, "null arg");
    struct Blk {
        int64_t src, clen, dst;
        uint32_t isize;
    };
    std::vector<Blk> bl;
    int64_t o = 0, tot = 0;
    while (o < len) {
        if (len - o < 18 || data[o] != 31 || data[o + 1] != 139 || data[o + 2] != 8 || !(data[o + 3] & 4))
            return pr_set_error(PR_ERR_ARG, "not a BGZF block");
        const int xlen = data[o + 10] | (data[o + 11] << 8);
        if (o + 12 + xlen > len) return pr_set_error(PR_ERR_ARG, "truncated BGZF header");
        int bsize = -1;
        for (int e = 0; e + 4 <= xlen;) {
            const uint8_t *x = data + o + 12 + e;
            const int sl = x[2] | (x[3] << 8);
            if (x[0] == 66 && x[1] == 67 && sl == 2 && e + 6 <= xlen) bsize = x[4] | (x[5] << 8);
            e += 4 + sl;
        }
        if (bsize < 0) return pr_set_error(PR_ERR_ARG, "BGZF block without BC field");
        const int64_t end = o + bsize + 1;
        if (end > len || bsize + 1 < 12 + xlen + 8) return pr_set_error(PR_ERR_ARG, "truncated BGZF block");
        const uint8_t *t = data + end - 4;
        const uint32_t isize = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
        bl.push_back(Blk{o + 12 + xlen, bsize + 1 - 12 - xlen - 8, tot, isize});
        tot += isize;
        o = end;
    }
    uint8_t *buf = (uint8_t *)std::malloc((size_t)(tot > 0 ? tot : 1));
    if (!buf) return pr_set_error(PR_ERR_ARG, "out of host memory");
    const int64_t nb = (int64_t)bl.size();
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    if (nb < 2) nt = 1;
    std::vector<int> fail((size_t)(nb ? nb : 1), 0);
    auto work = [&](int th) {
        for (int64_t b = th; b < nb; b += nt) {
            const Blk &k = bl[(size_t)b];
            if (k.isize == 0) continue;
            z_stream z;
            std::memset(&z, 0, sizeof z);
            if (inflateInit2(&z, -15) != Z_OK) { fail[b] = 1; continue; }
            z.next_in = const_cast<Bytef *>(data + k.src);
            z.avail_in = (uInt)k.clen;
            z.next_out = buf + k.dst;
            z.avail_out = k.isize;
            const int rc = inflate(&z, Z_FINISH);
            if (rc != Z_STREAM_END || z.avail_out != 0) fail[b] = 1;
            inflateEnd(&z);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    for (int64_t b = 0; b < nb; ++b)
        if (fail[b]) {
            std::free(buf);
            return pr_set_error(PR_ERR_ARG, "inflate failed (corrupt BGZF block)");
        }
    *out = buf;
    *out_len = tot;
    return 0;
}

// samtools sort (coordinate) of a BAM record stream (block_size-prefixed records, the
// part of an uncompressed BAM after its header): key (reference id with unmapped last,
// POS+1 or 0 when unmapped, reverse flag), stable in input order on equal keys — the
// order of proovread_amd/bamio.py:record_key + sort_bam.
extern "C" int pr_bam_sort_records(const uint8_t *recs, int64_t len, int n_threads, uint8_t **out, int64_t *out_len,
                                   int64_t *n_records) {
    if (!out || !out_len || (len && !recs)) return pr_set_error(PR_ERR_ARG, "null arg");
    std::vector<int64_t> off;
    for (int64_t o = 0; o < len;) {
        if (len - o < 4) return pr_set_error(PR_ERR_ARG, "truncated BAM record");
        int32_t bs;
        std::memcpy(&bs, recs + o, 4);
        if (bs < 32 || o + 4 + bs > len) return pr_set_error(PR_ERR_ARG, "bad BAM record size");
        off.push_back(o);
        o += 4 + (int64_t)bs;
    }
    const int64_t n = (int64_t)off.size();
    struct Key {
        uint64_t hi, lo;   // reference id (unmapped: 2^31), then (POS+1) << 1 | reverse
        int64_t i;         // input index: stable on equal keys
        bool operator<(const Key &o) const {
            return hi != o.hi ? hi < o.hi : (lo != o.lo ? lo < o.lo : i < o.i);
        }
    };
    std::vector<Key> key((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t *r = recs + off[(size_t)i] + 4;
        int32_t rid, pos;
        uint16_t flag;
        std::memcpy(&rid, r, 4);
        std::memcpy(&pos, r + 4, 4);
        std::memcpy(&flag, r + 14, 2);
        const uint64_t k0 = rid >= 0 ? (uint64_t)rid : (uint64_t)1 << 31;
        const uint64_t k1 = rid >= 0 ? (uint64_t)(uint32_t)(pos + 1) : 0;
        key[(size_t)i] = Key{k0, (k1 << 1) | ((flag >> 4) & 1u), i};
    }
    std::sort(key.begin(), key.end());
    uint8_t *buf = (uint8_t *)std::malloc((size_t)(len > 0 ? len : 1));
    if (!buf) return pr_set_error(PR_ERR_ARG, "out of host memory");
    std::vector<int64_t> dst((size_t)n + 1, 0);
    for (int64_t j = 0; j < n; ++j) {
        const int64_t i = key[(size_t)j].i;
        const int64_t sz = (i + 1 < n ? off[(size_t)i + 1] : len) - off[(size_t)i];
        dst[(size_t)j + 1] = dst[(size_t)j] + sz;
    }
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    if (n < 4096) nt = 1;
    auto copy = [&](int t) {
        for (int64_t j = n * t / nt; j < n * (t + 1) / nt; ++j) {
            const int64_t i = key[(size_t)j].i;
            std::memcpy(buf + dst[(size_t)j], recs + off[(size_t)i], (size_t)(dst[(size_t)j + 1] - dst[(size_t)j]));
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(copy, t);
    copy(0);
    for (auto &x : th) x.join();
    *out = buf;
    *out_len = len;
    if (n_records) *n_records = n;
    return 0;
}

// Perl's numification of an AS:Z string as proovread_amd/cns.py:parse_perl_number reads
// it: optional spaces, then [+-]?(digits[.digits][e[+-]digits] | .digits[e[+-]digits]), else 0
static double perl_number(const char *s, const char *e) {
    const char *p = s;
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\f' || *p == '\v')) ++p;
    const char *b = p;
    if (p < e && (*p == '+' || *p == '-')) ++p;
    const char *d0 = p;
    while (p < e && *p >= '0' && *p <= '9') ++p;
    bool ok = p > d0;
    if (ok) {
        if (p < e && *p == '.') {
            ++p;
            while (p < e && *p >= '0' && *p <= '9') ++p;
        }
    } else if (p + 1 < e && *p == '.' && p[1] >= '0' && p[1] <= '9') {
        ++p;
        while (p < e && *p >= '0' && *p <= '9') ++p;
        ok = true;
    }
    if (!ok) return 0.0;
    if (p < e && (*p == 'e' || *p == 'E')) {
        const char *q = p + 1;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        const char *q0 = q;
        while (q < e && *q >= '0' && *q <= '9') ++q;
        if (q > q0) p = q;
    }
    return std::strtod(std::string(b, p).c_str(), nullptr);
}

// BAM record stream -> the per-alignment arrays of the consensus stage (bam2cns's BAM
// reader, proovread_amd/bam2cns.py:bam_records + cns.py:pack_chunk): POS, AS, flags, SEQ as
// printed ("=ACMGRSVTWYHKDBN"), QUAL as phred+33 ('!' for a missing one), CIGAR ops.
// Records are walked once for their sizes, then decoded in parallel into the pools.
extern "C" int pr_bam_decode_alns(const uint8_t *recs, int64_t len, int n_threads, pr_bam_alns *out) {
    if (!out || (len && !recs)) return pr_set_error(PR_ERR_ARG, "null arg");
    std::memset(out, 0, sizeof *out);
    std::vector<int64_t> off;
    std::vector<int64_t> so(1, 0), co(1, 0);
    for (int64_t o = 0; o < len;) {
        if (len - o < 4) return pr_set_error(PR_ERR_ARG, "truncated BAM record");
        int32_t bs, l_seq;
        std::memcpy(&bs, recs + o, 4);
        if (bs < 32 || o + 4 + bs > len) return pr_set_error(PR_ERR_ARG, "bad BAM record size");
        const uint8_t *r = recs + o + 4;
        uint16_t n_cig;
        std::memcpy(&n_cig, r + 12, 2);
        std::memcpy(&l_seq, r + 16, 4);
        const int64_t need = 32 + (int64_t)r[8] + 4 * (int64_t)n_cig + (l_seq + 1) / 2 + l_seq;
        if (l_seq < 0 || need > bs) return pr_set_error(PR_ERR_ARG, "BAM record fields exceed its size");
        off.push_back(o);
        so.push_back(so.back() + l_seq);
        co.push_back(co.back() + n_cig);
        o += 4 + (int64_t)bs;
    }
    const int64_t n = (int64_t)off.size();
    auto alloc = [](size_t b) { return std::malloc(b ? b : 1); };
    out->n = n;
    out->rid = (int32_t *)alloc(4 * (size_t)n);
    out->pos1 = (int32_t *)alloc(4 * (size_t)n);
    out->score = (double *)alloc(8 * (size_t)n);
    out->flags = (uint8_t *)alloc((size_t)n);
    out->seq_off = (int64_t *)alloc(8 * (size_t)n);
    out->lseq = (int32_t *)alloc(4 * (size_t)n);
    out->cig_off = (int64_t *)alloc(8 * (size_t)n);
    out->ncig = (int32_t *)alloc(4 * (size_t)n);
    out->seq = (uint8_t *)alloc((size_t)so.back());
    out->qual = (uint8_t *)alloc((size_t)so.back());
    out->cig = (uint32_t *)alloc(4 * (size_t)co.back());
    out->seq_len = so.back();
    out->cig_len = co.back();
    if (!out->rid || !out->pos1 || !out->score || !out->flags || !out->seq_off || !out->lseq || !out->cig_off ||
        !out->ncig || !out->seq || !out->qual || !out->cig) {
        pr_bam_alns_free(out);
        return pr_set_error(PR_ERR_ARG, "out of host memory");
    }
    static const char NT16[] = "=ACMGRSVTWYHKDBN";
    std::vector<int> bad((size_t)(n ? n : 1), 0);
    auto work = [&](int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            const uint8_t *r = recs + off[(size_t)i] + 4;
            int32_t bs, rid, pos, l_seq;
            uint16_t n_cig;
            std::memcpy(&bs, recs + off[(size_t)i], 4);
            std::memcpy(&rid, r, 4);
            std::memcpy(&pos, r + 4, 4);
            std::memcpy(&n_cig, r + 12, 2);
            std::memcpy(&l_seq, r + 16, 4);
            const uint8_t *end = r + bs;
            const uint8_t *c = r + 32 + r[8];
            out->rid[i] = rid;
            out->pos1[i] = pos + 1;
            out->seq_off[i] = so[(size_t)i];
            out->lseq[i] = l_seq;
            out->cig_off[i] = co[(size_t)i];
            out->ncig[i] = n_cig;
            std::memcpy(out->cig + co[(size_t)i], c, 4 * (size_t)n_cig);
            const uint8_t *sb = c + 4 * n_cig;
            uint8_t *sd = out->seq + so[(size_t)i];
            for (int32_t k = 0; k < l_seq; ++k) sd[k] = (uint8_t)NT16[(sb[k >> 1] >> (4 * (1 - (k & 1)))) & 15];
            const uint8_t *qb = sb + (l_seq + 1) / 2;
            uint8_t *qd = out->qual + so[(size_t)i];
            uint8_t fl = l_seq == 0 ? PR_ALN_NO_SEQ : 0;
            if (l_seq && qb[0] == 0xFF) {
                fl |= PR_ALN_NO_QUAL;
                std::memset(qd, '!', (size_t)l_seq);
            } else {
                for (int32_t k = 0; k < l_seq; ++k) qd[k] = (uint8_t)(qb[k] + 33);
            }
            double score = 0.0;
            const uint8_t *a = qb + l_seq;
            while (a < end) {   // aux fields: the last AS tag wins
                if (end - a < 3) { bad[(size_t)i] = 1; break; }
                const bool as = a[0] == 'A' && a[1] == 'S';
                const char t = (char)a[2];
                a += 3;
                int64_t v = 0;
                const int sz = (t == 'c' || t == 'C') ? 1 : (t == 's' || t == 'S') ? 2 : (t == 'i' || t == 'I') ? 4 : 0;
                if (sz && a + sz > end) { bad[(size_t)i] = 1; break; }   // check before reading the value
                switch (t) {
                    case 'c': v = (int8_t)a[0]; break;
                    case 'C': v = a[0]; break;
                    case 's': { int16_t x; std::memcpy(&x, a, 2); v = x; break; }
                    case 'S': { uint16_t x; std::memcpy(&x, a, 2); v = x; break; }
                    case 'i': { int32_t x; std::memcpy(&x, a, 4); v = x; break; }
                    case 'I': { uint32_t x; std::memcpy(&x, a, 4); v = x; break; }
                    default: break;
                }
                if (sz) {
                    if (as) { score = (double)v; fl |= PR_ALN_HAS_SCORE; }
                    a += sz;
                } else if (t == 'A' || t == 'f') {
                    const int w = t == 'A' ? 1 : 4;
                    if (a + w > end) { bad[(size_t)i] = 1; break; }
                    if (as && t == 'f') {
                        float f;
                        std::memcpy(&f, a, 4);
                        score = (double)f;
                        fl |= PR_ALN_HAS_SCORE;
                    }
                    a += w;
                } else if (t == 'Z' || t == 'H') {
                    const uint8_t *z = a;
                    while (z < end && *z) ++z;
                    if (z >= end) { bad[(size_t)i] = 1; break; }
                    if (as) { score = perl_number((const char *)a, (const char *)z); fl |= PR_ALN_HAS_SCORE; }
                    a = z + 1;
                } else if (t == 'B') {
                    if (end - a < 5) { bad[(size_t)i] = 1; break; }
                    const char st = (char)a[0];
                    int32_t cnt;
                    std::memcpy(&cnt, a + 1, 4);
                    const int es = (st == 'c' || st == 'C') ? 1 : (st == 's' || st == 'S') ? 2 :
                                   (st == 'i' || st == 'I' || st == 'f') ? 4 : 0;
                    if (!es || cnt < 0 || a + 5 + (int64_t)cnt * es > end) { bad[(size_t)i] = 1; break; }
                    a += 5 + (int64_t)cnt * es;
                } else {
                    bad[(size_t)i] = 1;
                    break;
                }
            }
            out->score[i] = score;
            out->flags[i] = fl;
        }
    };
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    if (n < 4096) nt = 1;
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, n * t / nt, n * (t + 1) / nt);
    work(0, n / nt);
    for (auto &x : th) x.join();
    for (int64_t i = 0; i < n; ++i)
        if (bad[(size_t)i]) {
            pr_bam_alns_free(out);
            return pr_set_error(PR_ERR_SAM, "bad BAM aux field");
        }
    return 0;
}

extern "C" void pr_bam_alns_free(pr_bam_alns *a) {
    if (!a) return;
    void *p[] = {a->rid, a->pos1, a->score, a->flags, a->seq_off, a->lseq, a->cig_off, a->ncig, a->seq, a->qual, a->cig};
    for (void *x : p) std::free(x);
    std::memset(a, 0, sizeof *a);
}

// `samtools index` (bin/proovread:1343-1355) of a coordinate-sorted BAM file: the BAI of
// proovread_amd/bamio.py:index_bam — per reference the bins with their chunks (virtual
// offsets, adjacent chunks of one bin merged), the pseudo-bin 37450 (first/last offset,
// mapped/unmapped counts), the 16 kb linear index (empty windows take the previous one), and
// the count of records without coordinates.  Virtual offsets follow the BGZF reader: a
// position at the end of a block is the start of the next block.
extern "C" int pr_bam_index(const uint8_t *data, int64_t len, int n_threads, uint8_t **out, int64_t *out_len) {
    if (!out || !out_len || (len && !data)) return pr_set_error(PR_ERR_ARG, "null arg");
    // block table (compressed offset, uncompressed start) of the file
    std::vector<int64_t> coff, ustart;
    int64_t tot = 0;
    for (int64_t o = 0; o < len;) {
        if (len - o < 18 || data[o] != 31 || data[o + 1] != 139) return pr_set_error(PR_ERR_ARG, "not a BGZF block");
        const int xlen = data[o + 10] | (data[o + 11] << 8);
        int bsize = -1;
        for (int e = 0; e + 4 <= xlen && o + 12 + e + 4 <= len;) {
            const uint8_t *x = data + o + 12 + e;
            const int sl = x[2] | (x[3] << 8);
            if (x[0] == 66 && x[1] == 67 && sl == 2) bsize = x[4] | (x[5] << 8);
            e += 4 + sl;
        }
        // header (12 + xlen) + the CRC32 / ISIZE trailer (8) must fit in the block
        if (bsize < 0 || bsize + 1 < 12 + xlen + 8 || o + bsize + 1 > len) return pr_set_error(PR_ERR_ARG, "bad BGZF block");
        const uint8_t *t = data + o + bsize + 1 - 4;
        coff.push_back(o);
        ustart.push_back(tot);
        tot += (int64_t)((uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24));
        o += bsize + 1;
    }
    coff.push_back(len);
    ustart.push_back(tot);
    uint8_t *u = nullptr;
    int64_t ulen = 0;
    int rc = pr_bgzf_decompress(data, len, n_threads, &u, &ulen);
    if (rc) return rc;
    std::unique_ptr<uint8_t, void (*)(void *)> hold(u, std::free);
    // virtual offset of stream position p (monotone queries: block cursor)
    const size_t nblk = coff.size() - 1;   // real blocks; coff[nblk] = file length
    size_t cb = 0;
    auto voff = [&](int64_t p) -> uint64_t {
        while (cb < nblk && ustart[cb + 1] < p) ++cb;   // skip blocks that end before p
        if (cb < nblk && ustart[cb + 1] == p && ustart[cb + 1] > ustart[cb])
            return (uint64_t)coff[cb + 1] << 16;       // the end of a block reads as the next block's start
        return ((uint64_t)coff[cb] << 16) | (uint64_t)(p - ustart[cb]);
    };
    if (ulen < 12 || std::memcmp(u, "BAM\1", 4) != 0) return pr_set_error(PR_ERR_ARG, "not a BAM file");
    int32_t l_text, n_ref;
    std::memcpy(&l_text, u + 4, 4);
    int64_t p = 8 + (int64_t)l_text;
    if (l_text < 0 || p + 4 > ulen) return pr_set_error(PR_ERR_ARG, "truncated BAM header");
    std::memcpy(&n_ref, u + p, 4);
    p += 4;
    for (int32_t r = 0; r < n_ref; ++r) {
        int32_t ln;
        if (p + 4 > ulen) return pr_set_error(PR_ERR_ARG, "truncated BAM header");
        std::memcpy(&ln, u + p, 4);
        p += 8 + (int64_t)ln;
    }
    if (n_ref < 0 || p > ulen) return pr_set_error(PR_ERR_ARG, "truncated BAM header");
    struct Meta {
        bool any = false;
        uint64_t beg = 0, end = 0, mapped = 0, unmapped = 0;
    };
    std::vector<std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>>> bins((size_t)n_ref);
    std::vector<std::vector<uint64_t>> lin((size_t)n_ref);
    std::vector<Meta> meta((size_t)n_ref);
    uint64_t n_no_coor = 0;
    int32_t last_rid = -1, last_pos = -1;
    while (p < ulen) {
        if (ulen - p < 4) return pr_set_error(PR_ERR_ARG, "truncated BAM record");
        int32_t bs;
        std::memcpy(&bs, u + p, 4);
        if (bs < 32 || p + 4 + bs > ulen) return pr_set_error(PR_ERR_ARG, "bad BAM record size");
        const uint64_t v = voff(p);
        const uint8_t *r = u + p + 4;
        p += 4 + (int64_t)bs;
        const uint64_t ve = voff(p);
        int32_t rid, pos;
        uint16_t bin, n_cig, flag;
        std::memcpy(&rid, r, 4);
        std::memcpy(&pos, r + 4, 4);
        std::memcpy(&bin, r + 10, 2);
        std::memcpy(&n_cig, r + 12, 2);
        std::memcpy(&flag, r + 14, 2);
        if (rid < 0) {
            ++n_no_coor;
            continue;
        }
        if (rid >= n_ref) return pr_set_error(PR_ERR_ARG, "record reference id out of range");
        if (rid < last_rid || (rid == last_rid && pos < last_pos)) return pr_set_error(PR_ERR_ARG, "not coordinate-sorted");
        last_rid = rid;
        last_pos = pos;
        if (32 + (int64_t)r[8] + 4 * (int64_t)n_cig > bs) return pr_set_error(PR_ERR_ARG, "bad BAM record");
        int64_t span = 0;
        for (int k = 0; k < n_cig; ++k) {
            uint32_t op;
            std::memcpy(&op, r + 32 + r[8] + 4 * k, 4);
            const uint32_t c = op & 15;
            if (c == 0 || c == 2 || c == 3 || c == 7 || c == 8) span += op >> 4;
        }
        // hts_idx_push: a placed record without a position (POS 0 in SAM, pos -1 here) indexes
        // at 0; its end is at least one past its start
        const int64_t beg = pos < 0 ? 0 : (int64_t)pos;
        int64_t end = (int64_t)pos + (span ? span : 1);
        if (end < beg + 1) end = beg + 1;
        auto &ch = bins[(size_t)rid][bin];
        if (!ch.empty() && ch.back().second == v) ch.back().second = ve;
        else ch.emplace_back(v, ve);
        auto &li = lin[(size_t)rid];
        for (int64_t w = beg >> 14; w <= (end - 1) >> 14; ++w) {
            if ((int64_t)li.size() <= w) li.resize((size_t)w + 1, 0);
            if (li[(size_t)w] == 0) li[(size_t)w] = v;
        }
        Meta &m = meta[(size_t)rid];
        if (!m.any) {
            m.any = true;
            m.beg = v;
        }
        m.end = ve;
        if (flag & 4) ++m.unmapped;
        else ++m.mapped;
    }
    std::string o("BAI\1", 4);
    put<int32_t>(o, n_ref);
    for (int32_t rid = 0; rid < n_ref; ++rid) {
        const auto &b = bins[(size_t)rid];
        const Meta &m = meta[(size_t)rid];
        put<int32_t>(o, (int32_t)b.size() + (m.any ? 1 : 0));
        for (const auto &kv : b) {
            put<uint32_t>(o, kv.first);
            put<int32_t>(o, (int32_t)kv.second.size());
            for (const auto &c : kv.second) {
                put<uint64_t>(o, c.first);
                put<uint64_t>(o, c.second);
            }
        }
        if (m.any) {
            put<uint32_t>(o, 37450u);
            put<int32_t>(o, 2);
            put<uint64_t>(o, m.beg);
            put<uint64_t>(o, m.end);
            put<uint64_t>(o, m.mapped);
            put<uint64_t>(o, m.unmapped);
        }
        auto li = lin[(size_t)rid];
        for (size_t i = 1; i < li.size(); ++i)
            if (li[i] == 0) li[i] = li[i - 1];
        put<int32_t>(o, (int32_t)li.size());
        for (uint64_t x : li) put<uint64_t>(o, x);
    }
    put<uint64_t>(o, n_no_coor);
    *out = take(o, out_len);
    return *out ? 0 : pr_set_error(PR_ERR_ARG, "out of host memory");
}

extern "C" void pr_buffer_free(void *p) { std::free(p); }

// bam2cns:488's chimera lines (include/prgpu.h pr_fmt_chim_lines), each line written once into a
// growing buffer.  RATIO as Perl (and Python's '%.15g') prints it: std::to_chars(general, 15) is
// printf's %.15g (correctly rounded) without its per-call cost; nan / inf spelled as Python does.
extern "C" int pr_fmt_chim_lines(int32_t n_lr, const char *names, const int64_t *name_off, const int32_t *nchim,
                                 const int64_t *chim_off, const int32_t *chim, char **text, int64_t *len,
                                 int64_t *n_lines) {
    if (!text || !len || !n_lines || n_lr < 0 || (n_lr && (!names || !name_off || !nchim || !chim_off || !chim)))
        return -1;
    *text = nullptr;
    *len = 0;
    *n_lines = 0;
    int64_t lines = 0, cap = 1;
    for (int32_t i = 0; i < n_lr; ++i)
        if (nchim[i] > 0) lines += nchim[i], cap += (int64_t)nchim[i] * (name_off[i + 1] - name_off[i] + 48);
    char *out = static_cast<char *>(std::malloc((size_t)cap));
    if (!out) return -1;
    char *w = out;
    for (int32_t i = 0; i < n_lr; ++i) {
        const int32_t n = nchim[i];
        if (n <= 0) continue;
        const int64_t nl = name_off[i + 1] - name_off[i];
        for (int32_t j = 0; j < n; ++j) {
            const int32_t *r = chim + 4 * (chim_off[i] + j);
            std::memcpy(w, names + name_off[i], (size_t)nl);
            w += nl;
            *w++ = '\t';
            w = std::to_chars(w, w + 12, r[0]).ptr;
            *w++ = '\t';
            w = std::to_chars(w, w + 12, r[1]).ptr;
            *w++ = '\t';
            const double x = (double)r[2] / (double)r[3];
            if (std::isnan(x)) {
                std::memcpy(w, "nan", 3);
                w += 3;
            } else if (std::isinf(x)) {
                const int k = x > 0 ? 3 : 4;
                std::memcpy(w, x > 0 ? "inf" : "-inf", (size_t)k);
                w += k;
            } else {
                w = std::to_chars(w, w + 24, x, std::chars_format::general, 15).ptr;
            }
            *w++ = '\n';
        }
    }
    *w = 0;
    *text = out;
    *len = (int64_t)(w - out);
    *n_lines = lines;
    return 0;
}
