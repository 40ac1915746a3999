// The seed index built on the device (`bwa-proovread index`): the
// same tables as seed.cpp's pr_seed_index_build, byte for byte, from the long reads
// straight into the context's HBM (no host build, no index upload).
//
//   text   forward long reads, then the reverse complement of their concatenation,
//          each contig followed by SEP (5); one thread per forward base writes both
//          strands (read found by binary search over the read offsets)
//   keys   one thread per text position: the 12-mer code starting there (or NK when
//          the 12 bases are not all A/C/G/T) -> (key, position) pairs, and the k-mer
//          histogram (device atomics)
//   kpos   stable LSD radix sort of the pairs by key (rocPRIM, 25 key bits): every
//          k-mer's positions in ascending text order, as the host build leaves them
//   koff   exclusive scan of the histogram
//   kext   one thread per hit: the <= 28 bases after the 12-mer (2 bits each, stopping
//          at N / SEP) and their count << 56
//   cnt    j-mer counts, j = 11 .. 1: C_j(x) = sum_c C_{j+1}(4x + c) + #(runs of bases
//          ending in x), the run ends counted by one thread per N / SEP position
// HBM-bound integer work: ~n_text x (1 + 8 + 8 + 16) B for text, pairs and the sort's
// passes, ~12 B per hit for kpos / kext.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "seed_core.h"
#include "seed_index_dev.h"

namespace prgpu {

namespace {
constexpr uint8_t SEP = 5;
constexpr uint32_t NK = seedc::NK;
constexpr int KI = seedc::KI;
constexpr int KX = seedc::KX;

// Kernels over the whole text are grid-stride loops over a capped grid: a dispatch's grid is
// counted in work-items in 32 bits, and the text may exceed 2^32 positions.
// the long reads arrive as nt4 codes or ASCII (seedc::base_code); their nt4 codes are written
// back in place (the SW batch can take them from here: pr_sw_upload_gpu_seeds with lr_seq NULL)
__global__ void ix_text_kernel(uint8_t *lr_seq, const int64_t *lr_off, int n_lr, const int64_t *cstart,
                               int64_t l_pac, uint8_t *text) {
  const int64_t nt = l_pac > n_lr ? l_pac : n_lr;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nt; g += (int64_t)gridDim.x * blockDim.x) {
    if (g < l_pac) {
        int lo = 0, hi = n_lr - 1;   // read i: lr_off[i] <= g < lr_off[i + 1]
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (lr_off[mid] <= g) lo = mid; else hi = mid - 1;
        }
        const int i = lo;
        const int64_t p = g - lr_off[i], len = lr_off[i + 1] - lr_off[i];
        const uint8_t c = seedc::base_code(lr_seq[g]);
        lr_seq[g] = c;
        text[cstart[i] + p] = c;
        text[cstart[2 * (int64_t)n_lr - 1 - i] + (len - 1 - p)] = c < 4 ? (uint8_t)(3 - c) : 4;
    }
    if (g < n_lr) {   // separators
        const int64_t len = lr_off[g + 1] - lr_off[g];
        text[cstart[g] + len] = SEP;
        text[cstart[2 * (int64_t)n_lr - 1 - g] + len] = SEP;
    }
  }
}

// the 12-mer at every text position as a sort key (NK: none), no histogram: the hits' offsets
// come from the sorted keys (ix_koff_kernel; round 4 counted 290 M positions with global
// atomics, 10.8 ms of the 28 ms build at configs[1]).  The 12 bases from 4 dwords (the text
// buffer has 64 bytes of slack) aligned with v_alignbyte.
__global__ void ix_keys_kernel(const uint8_t *text, int64_t n, uint32_t *key, uint32_t *val) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint32_t code = 0;
    bool ok = p + KI <= n;
    if (ok) {
        const uint32_t *tw = reinterpret_cast<const uint32_t *>(text) + (p >> 2);
        const uint32_t sh = (uint32_t)(p & 3);
        const uint32_t w0 = tw[0], w1 = tw[1], w2 = tw[2], w3 = tw[3];
        const uint32_t x[3] = {__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                               __builtin_amdgcn_alignbyte(w3, w2, sh)};
#pragma unroll
        for (int j = 0; j < KI; ++j) {
            const uint32_t c = (x[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            ok &= c < 4u;
            code = (code << 2) | (c & 3u);
        }
    }
    key[p] = ok ? code : NK;
    val[p] = (uint32_t)p;
}

// koff from the sorted keys: koff[c] = the first slot with key >= c, for every c <= NK (each c
// written once: by the slot where the key steps past it, the codes after the last key by the
// last slot); then kc[c] = koff[c + 1] - koff[c] for the j-mer tables
__global__ void ix_koff_kernel(const uint32_t *skey, int64_t n, uint64_t *koff) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = skey[i] < NK ? skey[i] : NK;
    const int64_t kp = i > 0 ? (int64_t)(skey[i - 1] < NK ? skey[i - 1] : NK) : -1;
    for (int64_t c = kp + 1; c <= (int64_t)k; ++c) koff[c] = (uint64_t)i;
    if (i == n - 1)
        for (int64_t c = (int64_t)k + 1; c <= (int64_t)NK; ++c) koff[c] = (uint64_t)n;
}
__global__ void ix_kc_kernel(const uint64_t *koff, uint32_t *kc) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < (int64_t)NK) kc[c] = (uint32_t)(koff[c + 1] - koff[c]);
}

// the KX bases after the 12-mer at text position p: the 9 dwords around them loaded at once
// (independent loads from a random text position; the buffer's 64-byte slack covers the end),
// aligned with v_alignbyte, then the run up to the first N / separator / text end packed in
// registers (round 2: one dependent byte load per base, 41 ms at configs[1])
__device__ __forceinline__ uint64_t kext_at(const uint8_t *text, int64_t n, int64_t p12) {
    const int64_t p = p12 + KI;
    const uint32_t *tw = reinterpret_cast<const uint32_t *>(text) + (p >> 2);
    const uint32_t sh = (uint32_t)(p & 3);
    uint32_t w[9];
#pragma unroll
    for (int u = 0; u < 9; ++u) w[u] = tw[u];
    uint32_t x[7];
#pragma unroll
    for (int u = 0; u < 7; ++u) x[u] = __builtin_amdgcn_alignbyte(w[u + 1], w[u], sh);
    const int lim = n - p < KX ? (int)(n - p) : KX;
    uint64_t v = 0;
    int m = KX;
#pragma unroll
    for (int j = 0; j < KX; ++j) {
        const uint32_t c = (x[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        if (m == KX && (j >= lim || c > 3u)) m = j;
        if (m == KX) v |= (uint64_t)c << (2 * j);
    }
    return v | ((uint64_t)m << 56);
}

__global__ void ix_kext_kernel(const uint8_t *text, int64_t n, const uint32_t *kpos, const uint64_t *koff,
                               uint64_t *kext) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= (int64_t)koff[NK]) return;   // the hits: the sorted pairs with a valid key
    kext[r] = kext_at(text, n, (int64_t)kpos[r]);
}

// The positions whose 12 bases are all A/C/G/T, compacted in text order before the sort: the
// sort then takes 24 key bits (3 onesweep passes instead of 4 for 25, the 25th bit only ever
// separated the positions without a 12-mer) over fewer pairs (bwa-sr-2's mapping reference is
// ~70 % N).  off = exclusive scan of the valid flags; ckey / cval: the compacted pairs.
struct IxValid {
    __host__ __device__ uint32_t operator()(uint32_t k) const { return k < NK ? 1u : 0u; }
};
__global__ void ix_compact_kernel(const uint32_t *key, const uint32_t *off, int64_t n, uint32_t *ckey, uint32_t *cval) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t k = key[p];
    if (k < NK) {
        const uint32_t o = off[p];
        ckey[o] = k;
        cval[o] = (uint32_t)p;
    }
}

// chunked build (texts beyond one sort): the 12-mer histogram of the whole text
__global__ void ix_count_kernel(const uint8_t *text, int64_t n, uint32_t *kc) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p + KI <= n; p += (int64_t)gridDim.x * blockDim.x) {
        uint32_t code = 0;
        bool ok = true;
        for (int x = 0; x < KI; ++x) {
            const uint8_t c = text[p + x];
            ok &= c < 4;
            code = (code << 2) | (c & 3u);
        }
        if (ok) atomicAdd(&kc[code], 1u);
    }
}

// one chunk [c0, c0 + m): (key, position - c0) pairs and the chunk's histogram
__global__ void ix_chunk_keys_kernel(const uint8_t *text, int64_t n, int64_t c0, int64_t m, uint32_t *key,
                                     uint32_t *val, uint32_t *kcc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t p = c0 + i;
    uint32_t code = 0;
    bool ok = p + KI <= n;
    if (ok) {
        for (int x = 0; x < KI; ++x) {
            const uint8_t c = text[p + x];
            ok &= c < 4;
            code = (code << 2) | (c & 3u);
        }
    }
    key[i] = ok ? code : NK;
    val[i] = (uint32_t)i;
    if (ok) atomicAdd(&kcc[code], 1u);
}

// the chunk's sorted hits to their slots after the earlier chunks' hits of the same k-mer
__global__ void ix_chunk_scatter_kernel(const uint8_t *text, int64_t n, int64_t c0, const uint32_t *key,
                                        const uint32_t *val, const uint32_t *koffc, const uint64_t *kcur,
                                        uint32_t *kpos, uint64_t *kext) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)koffc[NK]) return;   // the valid keys sort first
    const uint32_t code = key[i];
    const uint64_t dst = kcur[code] + (uint64_t)(i - (int64_t)koffc[code]);
    const int64_t p = c0 + (int64_t)val[i];
    kpos[dst] = (uint32_t)p;
    kext[dst] = kext_at(text, n, p);
}

__global__ void ix_chunk_advance_kernel(uint64_t *kcur, const uint32_t *kcc) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < (int64_t)NK) kcur[x] += kcc[x];
}

// run ends: one thread per text position holding N / SEP; the j-mers (j < 12) that end
// just before it inside the run of bases are counted into cnt[j - 1]
// The j-mers of length j <= TAIL_LDS_J have 4^j <= 1024 counters, which every N / SEP position
// of a masked text hits (bwa-sr-2's mapping reference is ~70 % N: 3.3 ms of global atomics on a
// few addresses); they are counted in the workgroup's LDS and added to HBM once per block.
constexpr int TAIL_LDS_J = 5;
constexpr int TAIL_LDS_N = ((1 << (2 * (TAIL_LDS_J + 1))) - 4) / 3;   // 4 + 16 + ... + 4^TAIL_LDS_J
__global__ void __launch_bounds__(256) ix_tail_kernel(const uint8_t *text, int64_t n, uint32_t *const *cnt) {
    __shared__ uint32_t lc[TAIL_LDS_N];
    for (int k = threadIdx.x; k < TAIL_LDS_N; k += blockDim.x) lc[k] = 0u;
    __syncthreads();
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        if (text[p] <= 3) continue;
        uint32_t code = 0;
        for (int j = 1; j < KI; ++j) {
            if (p - j < 0) break;
            const uint8_t c = text[p - j];
            if (c > 3) break;
            code |= (uint32_t)c << (2 * (j - 1));   // T[p-j] is the first base of the j-mer
            if (j <= TAIL_LDS_J) atomicAdd(&lc[((1 << (2 * j)) - 4) / 3 + code], 1u);
            else atomicAdd(&cnt[j - 1][code], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < TAIL_LDS_N; k += blockDim.x) {
        const uint32_t v = lc[k];
        if (!v) continue;
        int j = 1;
        while (k >= ((1 << (2 * (j + 1))) - 4) / 3) ++j;   // table j holds [(4^j - 4) / 3, (4^(j+1) - 4) / 3)
        atomicAdd(&cnt[j - 1][k - ((1 << (2 * j)) - 4) / 3], v);
    }
}

// C_j(x) += sum_c C_{j+1}(4x + c)
__global__ void ix_jmer_kernel(uint32_t *cj, const uint32_t *cn, int64_t nj) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= nj) return;
    const uint4 v = reinterpret_cast<const uint4 *>(cn)[x];
    cj[x] += v.x + v.y + v.z + v.w;
}

inline unsigned blocks_for(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }
// grid-stride kernels: at most 2^22 workgroups (2^30 work-items per dispatch)
inline unsigned blocks_capped(int64_t n, int t) {
    const int64_t b = (n + t - 1) / t;
    return (unsigned)(b < 1 ? 1 : (b > ((int64_t)1 << 22) ? ((int64_t)1 << 22) : b));
}
}  // namespace

#define IXCHK(x)                                   \
    do {                                           \
        const hipError_t e_ = (x);                 \
        if (e_ != hipSuccess) return (int)e_;      \
    } while (0)

int seed_index_device_build(const SeedIndexBuild &B, hipStream_t s) {
    const int64_t n = B.n_text;
    // text
    if (B.l_pac > 0 || B.n_lr > 0) {
        const int64_t nt = B.l_pac > B.n_lr ? B.l_pac : B.n_lr;
        hipLaunchKernelGGL(ix_text_kernel, dim3(blocks_capped(nt, 256)), dim3(256), 0, s, B.lr_seq, B.lr_off, B.n_lr,
                           B.cstart, B.l_pac, B.text);
        IXCHK(hipGetLastError());
    }
    IXCHK(hipMemsetAsync(B.kc, 0, ((size_t)NK + 1) * 4, s));
    if (n <= B.chunk) {
        // one sort: 12-mer keys + histogram, koff = exclusive scan, stable sort of (key,
        // position) by key (positions ascend within a k-mer) straight into kpos, then kext
        if (n > 0) {
            hipLaunchKernelGGL(ix_keys_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, B.text, n, B.key0, B.val0);
            IXCHK(hipGetLastError());
            // the valid pairs compacted (keys into the kext buffer, free until the kext pass), then
            // sorted by their 24 key bits into key0 / kpos
            size_t tb = B.temp_bytes;
            auto vit = rocprim::make_transform_iterator(B.key0, IxValid{});
            IXCHK(rocprim::exclusive_scan(B.temp, tb, vit, B.key1, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
            uint32_t *ckey = reinterpret_cast<uint32_t *>(B.kext);
            hipLaunchKernelGGL(ix_compact_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, B.key0, B.key1, n, ckey, B.val0);
            IXCHK(hipGetLastError());
            uint32_t last[2] = {0u, 0u};   // the scan's last entry and the last key: the valid count
            IXCHK(hipMemcpyAsync(&last[0], B.key1 + (n - 1), 4, hipMemcpyDeviceToHost, s));
            IXCHK(hipMemcpyAsync(&last[1], B.key0 + (n - 1), 4, hipMemcpyDeviceToHost, s));
            IXCHK(hipStreamSynchronize(s));
            const int64_t nv = (int64_t)last[0] + (last[1] < NK ? 1 : 0);
            tb = B.temp_bytes;
            if (nv > 0) IXCHK(rocprim::radix_sort_pairs(B.temp, tb, ckey, B.key0, B.val0, B.kpos, (size_t)nv, 0u, 24u, s));
            if (nv > 0) {
                hipLaunchKernelGGL(ix_koff_kernel, dim3(blocks_for(nv, 256)), dim3(256), 0, s, B.key0, nv, B.koff);
                IXCHK(hipGetLastError());
            } else {
                IXCHK(hipMemsetAsync(B.koff, 0, ((size_t)NK + 1) * 8, s));
            }
            hipLaunchKernelGGL(ix_kc_kernel, dim3(blocks_for((int64_t)NK, 256)), dim3(256), 0, s, B.koff, B.kc);
            IXCHK(hipGetLastError());
            hipLaunchKernelGGL(ix_kext_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, B.text, n, B.kpos, B.koff,
                               B.kext);
            IXCHK(hipGetLastError());
        } else {
            IXCHK(hipMemsetAsync(B.koff, 0, ((size_t)NK + 1) * 8, s));
        }
    } else {
        // chunks of B.chunk positions (a divisor of 2^32, so one starts at 2^32): the global
        // histogram and koff first, then per chunk a sort and a scatter of its hits behind the
        // earlier chunks' (kcur); ksplit = kcur when the chunk at 2^32 begins
        hipLaunchKernelGGL(ix_count_kernel, dim3(blocks_capped(n, 256)), dim3(256), 0, s, B.text, n, B.kc);
        IXCHK(hipGetLastError());
        size_t tb = B.temp_bytes;
        IXCHK(rocprim::exclusive_scan(B.temp, tb, B.kc, B.koff, (uint64_t)0, (size_t)NK + 1, rocprim::plus<uint64_t>(), s));
        IXCHK(hipMemcpyAsync(B.kcur, B.koff, (size_t)NK * 8, hipMemcpyDeviceToDevice, s));
        for (int64_t c0 = 0; c0 < n; c0 += B.chunk) {
            const int64_t m = n - c0 < B.chunk ? n - c0 : B.chunk;
            if (c0 == (int64_t)seedc::POS_PAGE && B.ksplit)
                IXCHK(hipMemcpyAsync(B.ksplit, B.kcur, (size_t)NK * 8, hipMemcpyDeviceToDevice, s));
            IXCHK(hipMemsetAsync(B.kcc, 0, ((size_t)NK + 1) * 4, s));
            hipLaunchKernelGGL(ix_chunk_keys_kernel, dim3(blocks_for(m, 256)), dim3(256), 0, s, B.text, n, c0, m,
                               B.key0, B.val0, B.kcc);
            IXCHK(hipGetLastError());
            tb = B.temp_bytes;
            IXCHK(rocprim::exclusive_scan(B.temp, tb, B.kcc, B.koffc, 0u, (size_t)NK + 1, rocprim::plus<uint32_t>(), s));
            tb = B.temp_bytes;
            IXCHK(rocprim::radix_sort_pairs(B.temp, tb, B.key0, B.key1, B.val0, B.val1, (size_t)m, 0u, 25u, s));
            hipLaunchKernelGGL(ix_chunk_scatter_kernel, dim3(blocks_for(m, 256)), dim3(256), 0, s, B.text, n, c0, B.key1,
                               B.val1, B.koffc, B.kcur, B.kpos, B.kext);
            IXCHK(hipGetLastError());
            hipLaunchKernelGGL(ix_chunk_advance_kernel, dim3(blocks_for((int64_t)NK, 256)), dim3(256), 0, s, B.kcur,
                               B.kcc);
            IXCHK(hipGetLastError());
        }
    }
    // j-mer count tables: run ends first, then the children's sums from j = 11 down
    for (int j = 1; j < KI; ++j) IXCHK(hipMemsetAsync(B.cnt[j - 1], 0, ((size_t)1 << (2 * j)) * 4, s));
    if (n > 0) {
        // (a grid of 8192 blocks striding over the text: each block's LDS counts flushed once)
        const unsigned tb = blocks_capped(n, 256) < 8192u ? blocks_capped(n, 256) : 8192u;
        hipLaunchKernelGGL(ix_tail_kernel, dim3(tb), dim3(256), 0, s, B.text, n, B.cnt_dev);
        IXCHK(hipGetLastError());
    }
    for (int j = KI - 1; j >= 1; --j) {
        const uint32_t *cn = j == KI - 1 ? B.kc : B.cnt[j];
        const int64_t nj = (int64_t)1 << (2 * j);
        hipLaunchKernelGGL(ix_jmer_kernel, dim3(blocks_for(nj, 256)), dim3(256), 0, s, B.cnt[j - 1], cn, nj);
        IXCHK(hipGetLastError());
    }
    return 0;
}

// the text 16 bases per word, 4 bits each (base k of word w at bits 4k..4k+3; past the text: SEP),
// for the device occurrence table's 16-base match-length comparisons
__global__ void ix_pack4_kernel(const uint8_t *text, int64_t n_text, uint64_t *text4, int64_t n_words) {
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words; w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t v = 0;
        for (int k = 0; k < 16; ++k) {
            const int64_t x = w * 16 + k;
            const uint64_t c = x < n_text ? (uint64_t)text[x] : (uint64_t)SEP;
            v |= c << (4 * k);
        }
        text4[w] = v;
    }
}
// (8 padding words: the occurrence table's match-length walk loads 5 words at a time from any
// word a match can reach, seed_kernels.hip build_occ_wave)
int64_t ix_pack4_words(int64_t n_text) { return n_text / 16 + 8; }
int ix_pack4_launch(const uint8_t *text, int64_t n_text, uint64_t *text4, hipStream_t s) {
    const int64_t nw = ix_pack4_words(n_text);
    int64_t blocks = (nw + 255) / 256;
    blocks = blocks < (1 << 20) ? (blocks > 0 ? blocks : 1) : (1 << 20);
    hipLaunchKernelGGL(ix_pack4_kernel, dim3((unsigned)blocks), dim3(256), 0, s, text, n_text, text4, nw);
    return (int)hipGetLastError();
}

// bytes of rocPRIM temporary storage for sorts of `chunk` text positions
size_t seed_index_temp_bytes(int64_t chunk) {
    size_t a = 0, b = 0, c = 0;
    (void)rocprim::exclusive_scan(nullptr, a, (uint32_t *)nullptr, (uint64_t *)nullptr, (uint64_t)0, (size_t)NK + 1,
                                  rocprim::plus<uint64_t>());
    (void)rocprim::exclusive_scan(nullptr, c, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)NK + 1,
                                  rocprim::plus<uint32_t>());
    (void)rocprim::radix_sort_pairs(nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                    (uint32_t *)nullptr, (size_t)(chunk > 0 ? chunk : 1), 0u, 25u);
    size_t d = 0;   // the valid-position scan of the one-sort build
    (void)rocprim::exclusive_scan(nullptr, d, rocprim::make_transform_iterator((uint32_t *)nullptr, IxValid{}),
                                  (uint32_t *)nullptr, 0u, (size_t)(chunk > 0 ? chunk : 1), rocprim::plus<uint32_t>());
    return std::max(std::max(a, d), std::max(b, c)) + 256;
}

}  // namespace prgpu
