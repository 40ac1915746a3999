// Short-read input (bin/proovread:1293: the short-read files are read as one stream, `cat
// $or_files`, and cut into chunks by SeqChunker): one native pass over a FASTQ stream of plain
// 4-line records instead of the host's numpy passes (newline search, record checks, a byte mask
// and its running sum, a table lookup: ~0.85 s for configs[1]'s 230 MB, a third of the whole
// correction loop).  The accepted input is exactly the numpy path's: '@' first, '\n' last, no
// '\r' anywhere, every record `@...\n SEQ\n +...\n QUAL\n` with QUAL as long as SEQ; anything
// else returns PR_ERR_ARG and the caller takes the general record parser (FASTA, multi-line).
#include <cstdint>
#include <cstring>

#include "../../include/prgpu.h"

namespace {
// the end (index of the '\n') of the line starting at p, or -1
inline int64_t line_end(const uint8_t *d, int64_t n, int64_t p) {
    const void *q = memchr(d + p, '\n', (size_t)(n - p));
    return q ? (int64_t)((const uint8_t *)q - d) : -1;
}

// one record from p: its sequence line [s0, s1) and the start of the next record, or false
inline bool record(const uint8_t *d, int64_t n, int64_t p, int64_t &s0, int64_t &s1, int64_t &next) {
    if (d[p] != '@') return false;
    const int64_t h = line_end(d, n, p);
    if (h < 0) return false;
    s0 = h + 1;
    if (s0 >= n) return false;
    s1 = line_end(d, n, s0);
    if (s1 < 0 || s1 + 1 >= n || d[s1 + 1] != '+') return false;
    const int64_t pl = line_end(d, n, s1 + 1);
    if (pl < 0) return false;
    const int64_t q = line_end(d, n, pl + 1);
    if (q < 0 || q - (pl + 1) != s1 - s0) return false;
    next = q + 1;
    return true;
}
}  // namespace

extern "C" int pr_fastq4_scan(const uint8_t *d, int64_t n, int64_t *n_rec, int64_t *n_bases) {
    if (!d || !n_rec || !n_bases || n <= 0) return PR_ERR_ARG;
    if (d[0] != '@' || d[n - 1] != '\n' || memchr(d, '\r', (size_t)n)) return PR_ERR_ARG;
    int64_t r = 0, b = 0, p = 0, s0, s1, next;
    while (p < n) {
        if (!record(d, n, p, s0, s1, next)) return PR_ERR_ARG;
        ++r;
        b += s1 - s0;
        p = next;
    }
    *n_rec = r;
    *n_bases = b;
    return 0;
}

extern "C" int pr_fastq4_fill(const uint8_t *d, int64_t n, const uint8_t *table256, int64_t *starts, int64_t *off,
                              uint8_t *pool) {
    if (!d || !table256 || !starts || !off || !pool || n <= 0) return PR_ERR_ARG;
    int64_t r = 0, p = 0, s0, s1, next, o = 0;
    off[0] = 0;
    while (p < n) {
        if (!record(d, n, p, s0, s1, next)) return PR_ERR_ARG;
        starts[r] = p;
        for (int64_t x = s0; x < s1; ++x) pool[o++] = table256[d[x]];
        off[++r] = o;
        p = next;
    }
    return 0;
}
