// dict.hip — dense PC-id dictionary, presence marking and byte-map set algebra.
//
// The corpus' distinct PCs (= the union every `total = Union(total, cov)`
// fold of the reference computes: syz-manager/manager.go:610,
// syz-manager/html.go:72-79, cover/cover_test.go:182-185) are held as a uint8
// presence map over a PC window [pc_lo, pc_lo + pc_span).  A byte per PC
// (rather than a bit) makes marking a plain idempotent store (no atomics) and
// makes the cross-GPU merge an RCCL uint8 MAX all-reduce (RCCL has no OR).
// The dictionary packs the map into 32-PC words and an exclusive popcount
// prefix, interleaved as one u64 per word (prefix | bits << 32), so a PC's
// dense id is ONE 8-byte gather + a popcount (common.h dense_id).
#include "common.h"

#include <algorithm>

namespace syz {

__global__ void mark_kernel(const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
                            const uint32_t *__restrict__ pcs, size_t nseg,
                            uint8_t *__restrict__ pres, uint32_t pc_lo, uint64_t pc_span,
                            uint32_t *__restrict__ err) {
    for (size_t s = blockIdx.x; s < nseg; s += gridDim.x) {
        const uint64_t b = off[s];
        const uint64_t n = len ? len[s] : off[s + 1] - b;
        for (uint64_t k = threadIdx.x; k < n; k += blockDim.x) {
            const uint32_t pc = pcs[b + k];
            const uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
            if (pc < pc_lo || o >= pc_span) {
                *err = 1u;
                continue;
            }
            if (pres[o] == 0) pres[o] = 1;
        }
    }
}

// Contiguous corpus (lengths from offsets): mark is a flat stream over
// pcs[off[0] .. off[n]) with 16-byte vector loads (head/tail scalar).
__device__ __forceinline__ void mark_one(uint8_t *__restrict__ pres, uint32_t pc, uint32_t pc_lo,
                                         uint64_t pc_span, uint32_t *__restrict__ err) {
    const uint64_t o = (uint64_t)(uint32_t)(pc - pc_lo);
    if (pc < pc_lo || o >= pc_span) {
        *err = 1u;
        return;
    }
    if (pres[o] == 0) pres[o] = 1;
}

__global__ void mark_flat_kernel(const uint64_t *__restrict__ off, size_t nseg,
                                 const uint32_t *__restrict__ pcs, uint8_t *__restrict__ pres,
                                 uint32_t pc_lo, uint64_t pc_span, uint32_t *__restrict__ err) {
    const uint64_t start = off[0], end = off[nseg];
    // first 16-B aligned element at or after start
    const uint64_t a0 = (start + 3) & ~3ull;
    const uint64_t head_end = a0 < end ? a0 : end;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    if (tid < head_end - start) mark_one(pres, pcs[start + tid], pc_lo, pc_span, err);
    const uint64_t nvec = end > a0 ? (end - a0) / 4 : 0;
    const uint4 *v = (const uint4 *)(pcs + a0);
    for (uint64_t i = tid; i < nvec; i += nthr) {
        const uint4 x = v[i];
        mark_one(pres, x.x, pc_lo, pc_span, err);
        mark_one(pres, x.y, pc_lo, pc_span, err);
        mark_one(pres, x.z, pc_lo, pc_span, err);
        mark_one(pres, x.w, pc_lo, pc_span, err);
    }
    const uint64_t tail = a0 + nvec * 4;
    if (end > tail && tid < end - tail) mark_one(pres, pcs[tail + tid], pc_lo, pc_span, err);
}

// Bit-packed presence (8x smaller than the byte map, so the hot part of the
// window stays L2-resident): 16-B vector stream of PCs, the four word tests
// issued together, atomicOr only for bits not yet set.
__device__ __forceinline__ bool in_window(uint32_t pc, uint32_t pc_lo, uint64_t pc_span,
                                          uint64_t *o) {
    *o = (uint64_t)(uint32_t)(pc - pc_lo);
    return pc >= pc_lo && *o < pc_span;
}

__device__ __forceinline__ void mark_bit(uint32_t *__restrict__ bits, uint32_t pc, uint32_t pc_lo,
                                         uint64_t pc_span, uint32_t *__restrict__ err) {
    uint64_t o;
    if (!in_window(pc, pc_lo, pc_span, &o)) {
        *err = 1u;
        return;
    }
    const uint32_t m = 1u << (o & 31);
    if (!(bits[o >> 5] & m)) atomicOr(&bits[o >> 5], m);
}

// Bitmap set algebra on u32 words + popcount of the result.
__global__ __launch_bounds__(256) void bitmap_op_kernel(int op, uint32_t *__restrict__ dst,
                                                        const uint32_t *__restrict__ src,
                                                        uint64_t nwords,
                                                        unsigned long long *__restrict__ pop) {
    // 16-byte words per lane; popcount reduced per block, one atomic per block
    __shared__ uint32_t s_part[256 / 64];
    uint32_t cnt = 0;
    auto f = [op](uint32_t a, uint32_t b) {
        return op == 0 ? (a | b) : op == 1 ? (a & b) : op == 2 ? (a & ~b) : (a ^ b);
    };
    const bool al = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
    const uint64_t n4 = al ? nwords / 4 : 0;
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const uint4 a = d4[i], b = s4[i];
        const uint4 r = make_uint4(f(a.x, b.x), f(a.y, b.y), f(a.z, b.z), f(a.w, b.w));
        d4[i] = r;
        cnt += __popc(r.x) + __popc(r.y) + __popc(r.z) + __popc(r.w);
    }
    for (uint64_t i = n4 * 4 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
         i += stride) {
        const uint32_t r = f(dst[i], src[i]);
        dst[i] = r;
        cnt += __popc(r);
    }
    if (pop) {
        cnt = wave_sum(cnt);
        if (__lane_id() == 0) s_part[threadIdx.x >> 6] = cnt;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t t = s_part[0] + s_part[1] + s_part[2] + s_part[3];
            if (t) atomicAdd(pop, (unsigned long long)t);
        }
    }
}

// Pass A: each thread packs WPT consecutive 32-byte groups into words,
// writes {in-block exclusive prefix | bits << 32}, block total -> bsum[blk].
constexpr int DICT_THREADS = 256, DICT_WPT = 4, DICT_WPB = DICT_THREADS * DICT_WPT;

__device__ __forceinline__ uint32_t pack32(const uint8_t *__restrict__ p, uint64_t avail) {
    uint32_t bits = 0;
    if (avail >= 32) {
        const uint4 a = *(const uint4 *)p;
        const uint4 b = *(const uint4 *)(p + 16);
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int q = 0; q < 8; q++) {
#pragma unroll
            for (int by = 0; by < 4; by++) bits |= (((w[q] >> (8 * by)) & 0xFFu) != 0) << (q * 4 + by);
        }
    } else {
        for (uint64_t i = 0; i < avail; i++) bits |= (uint32_t)(p[i] != 0) << i;
    }
    return bits;
}

__global__ __launch_bounds__(DICT_THREADS) void dict_pass_a(const uint8_t *__restrict__ pres,
                                                             uint64_t span, uint64_t nwords,
                                                             uint64_t *__restrict__ tab,
                                                             uint32_t *__restrict__ bsum) {
    __shared__ uint32_t tmp[DICT_THREADS / 64 + 1];
    const uint64_t w0 = (uint64_t)blockIdx.x * DICT_WPB + (uint64_t)threadIdx.x * DICT_WPT;
    uint32_t bits[DICT_WPT], cnt = 0;
#pragma unroll
    for (int q = 0; q < DICT_WPT; q++) {
        const uint64_t w = w0 + q;
        bits[q] = 0;
        if (w < nwords) {
            const uint64_t base = w * 32;
            bits[q] = pack32(pres + base, span - base);
        }
        cnt += __popc(bits[q]);
    }
    uint32_t total;
    uint32_t pre = block_excl_scan<DICT_THREADS>(cnt, tmp, &total);
#pragma unroll
    for (int q = 0; q < DICT_WPT; q++) {
        const uint64_t w = w0 + q;
        if (w < nwords) tab[w] = (uint64_t)pre | ((uint64_t)bits[q] << 32);
        pre += __popc(bits[q]);
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// Bitmap variant of pass A (words already packed).
__global__ __launch_bounds__(DICT_THREADS) void dict_pass_a_bits(const uint32_t *__restrict__ bm,
                                                                  uint64_t nwords,
                                                                  uint64_t *__restrict__ tab,
                                                                  uint32_t *__restrict__ bsum) {
    __shared__ uint32_t tmp[DICT_THREADS / 64 + 1];
    const uint64_t w0 = (uint64_t)blockIdx.x * DICT_WPB + (uint64_t)threadIdx.x * DICT_WPT;
    uint32_t bits[DICT_WPT], cnt = 0;
#pragma unroll
    for (int q = 0; q < DICT_WPT; q++) {
        const uint64_t w = w0 + q;
        bits[q] = w < nwords ? bm[w] : 0u;
        cnt += __popc(bits[q]);
    }
    uint32_t total;
    uint32_t pre = block_excl_scan<DICT_THREADS>(cnt, tmp, &total);
#pragma unroll
    for (int q = 0; q < DICT_WPT; q++) {
        const uint64_t w = w0 + q;
        if (w < nwords) tab[w] = (uint64_t)pre | ((uint64_t)bits[q] << 32);
        pre += __popc(bits[q]);
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// Pass B: exclusive scan of block sums in one workgroup (chunks of 1024).
__global__ __launch_bounds__(1024) void dict_pass_b(uint32_t *__restrict__ bsum, uint64_t nblk,
                                                     uint32_t *__restrict__ n_ids) {
    __shared__ uint32_t tmp[1024 / 64 + 1];
    uint32_t carry = 0;
    for (uint64_t c = 0; c < nblk; c += 1024) {
        const uint64_t i = c + threadIdx.x;
        const uint32_t v = i < nblk ? bsum[i] : 0u;
        uint32_t total;
        const uint32_t p = block_excl_scan<1024>(v, tmp, &total);
        if (i < nblk) bsum[i] = carry + p;
        carry += total;
    }
    if (threadIdx.x == 0) *n_ids = carry;
}

// Pass C: add block offsets.
__global__ void dict_pass_c(uint64_t *__restrict__ tab, uint64_t nwords,
                            const uint32_t *__restrict__ bsum) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = tab[w];
        tab[w] = e + bsum[w / DICT_WPB];  // no carry into bits: prefix < 2^32
    }
}

// `drop`: the value Union drops (cover.go:97): PC 0xFFFFFFFF, or its KEY in
// key mode.  It is the largest value of the list either way (the key map is
// monotone), so leaving it out never leaves a hole.
__global__ void dict_to_list_kernel(const uint64_t *__restrict__ tab, uint64_t nwords,
                                    uint32_t pc_lo, uint32_t drop, uint32_t *__restrict__ out,
                                    uint32_t *__restrict__ n_out) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = tab[w];
        uint32_t bits = (uint32_t)(e >> 32);
        uint32_t pos = (uint32_t)e;
        while (out && bits) {
            const int b = __ffs(bits) - 1;
            bits &= bits - 1;
            const uint32_t pc = pc_lo + (uint32_t)(w * 32 + b);
            if (out && pc != drop) out[pos] = pc;  // Union drops the sentinel (cover.go:97)
            pos++;
        }
        if (w == nwords - 1) {
            // total = prefix of the last word + its popcount; minus sentinel
            uint32_t total = (uint32_t)e + __popc((uint32_t)(e >> 32));
            const uint64_t last_off = (uint64_t)(uint32_t)(drop - pc_lo);
            if (last_off / 32 == w && ((e >> 32) >> (last_off & 31)) & 1u) total -= 1;
            *n_out = total;
        }
    }
}

// Byte-map set algebra: 16 bytes per lane, coalesced; popcount of nonzero
// result bytes accumulated per wave then one atomic per wave.
__global__ void bytemap_op_kernel(int op, uint8_t *__restrict__ dst,
                                  const uint8_t *__restrict__ src, uint64_t nvec,
                                  unsigned long long *__restrict__ pop) {
    uint32_t cnt = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 d = ((const uint4 *)dst)[i];
        const uint4 s = ((const uint4 *)src)[i];
        uint32_t dv[4] = {d.x, d.y, d.z, d.w}, sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            // normalise bytes to 0/1 so AND/XOR/ANDNOT are set operations
            uint32_t a = dv[q], b = sv[q];
            uint32_t an = 0, bn = 0;
#pragma unroll
            for (int by = 0; by < 4; by++) {
                an |= (((a >> (8 * by)) & 0xFF) != 0) << (8 * by);
                bn |= (((b >> (8 * by)) & 0xFF) != 0) << (8 * by);
            }
            uint32_t r;
            switch (op) {
            case 0: r = an | bn; break;
            case 1: r = an & bn; break;
            case 2: r = an & ~bn; break;
            default: r = an ^ bn; break;
            }
            dv[q] = r;
            cnt += __popc(r);
        }
        ((uint4 *)dst)[i] = make_uint4(dv[0], dv[1], dv[2], dv[3]);
    }
    if (pop) {
        cnt = wave_sum(cnt);
        if (__lane_id() == 0 && cnt) atomicAdd(pop, (unsigned long long)cnt);
    }
}

__global__ void bytemap_tail_kernel(int op, uint8_t *__restrict__ dst,
                                    const uint8_t *__restrict__ src, uint64_t start, uint64_t n,
                                    unsigned long long *__restrict__ pop) {
    uint64_t i = start + threadIdx.x;
    uint32_t c = 0;
    if (i < n) {
        uint8_t a = dst[i] != 0, b = src[i] != 0, r;
        switch (op) {
        case 0: r = a | b; break;
        case 1: r = a & b; break;
        case 2: r = a & !b; break;
        default: r = a ^ b; break;
        }
        dst[i] = r;
        c = r;
    }
    if (pop) {
        c = wave_sum(c);
        if (__lane_id() == 0 && c) atomicAdd(pop, (unsigned long long)c);
    }
}

}  // namespace syz

using namespace syz;

extern "C" int syzcov_dev_mark(const uint64_t *off, const uint32_t *len, const uint32_t *pcs,
                               size_t nseg, uint8_t *pres, uint32_t pc_lo, uint64_t pc_span,
                               uint32_t *err_flag, void *stream) {
    if (nseg == 0) return 0;
    if (!off || !pcs || !pres || !err_flag) return SYZCOV_EINVAL;
    if (!len)  // contiguous CSR: one flat vectorised stream
        hipLaunchKernelGGL(mark_flat_kernel, dim3(256 * 16), dim3(256), 0, (hipStream_t)stream,
                           off, nseg, pcs, pres, pc_lo, pc_span, err_flag);
    else
        hipLaunchKernelGGL(mark_kernel, dim3(grid_for(nseg, 1, 8192)), dim3(256), 0,
                           (hipStream_t)stream, off, len, pcs, nseg, pres, pc_lo, pc_span,
                           err_flag);
    SYZ_LAUNCH_CHECK();
    return 0;
}




extern "C" int syzcov_dev_bitmap_op(int op, uint32_t *dst, const uint32_t *src, uint64_t nwords,
                                    uint64_t *popcount_out, void *stream) {
    if (op < 0 || op > 3 || !dst || !src) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long *pop = (unsigned long long *)popcount_out;
    if (pop) SYZ_HIP(hipMemsetAsync(pop, 0, sizeof(uint64_t), s));
    if (nwords) {
        hipLaunchKernelGGL(bitmap_op_kernel, dim3(grid_for((nwords + 3) / 4, 256, 1024)), dim3(256),
                           0, s, op,
                           dst, src, nwords, pop);
        SYZ_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" int syzcov_dev_dict_build_bits(const uint32_t *bits, uint64_t pc_span, uint64_t *tab,
                                          uint32_t *n_ids, void *ws, void *stream) {
    if (!bits || !tab || !n_ids || !ws || pc_span == 0 || pc_span > (1ull << 32))
        return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t nwords = (pc_span + 31) / 32;
    const uint64_t nblk = (nwords + DICT_WPB - 1) / DICT_WPB;
    uint32_t *bsum = (uint32_t *)ws;
    hipLaunchKernelGGL(dict_pass_a_bits, dim3((unsigned)nblk), dim3(DICT_THREADS), 0, s, bits,
                       nwords, tab, bsum);
    hipLaunchKernelGGL(dict_pass_b, dim3(1), dim3(1024), 0, s, bsum, nblk, n_ids);
    hipLaunchKernelGGL(dict_pass_c, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0, s, tab,
                       nwords, bsum);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" size_t syzcov_dev_dict_ws_size(uint64_t pc_span) {
    const uint64_t nwords = (pc_span + 31) / 32;
    const uint64_t nblk = (nwords + DICT_WPB - 1) / DICT_WPB;
    return align_up(nblk * sizeof(uint32_t), 256);
}

extern "C" int syzcov_dev_dict_build(const uint8_t *pres, uint64_t pc_span, uint64_t *tab,
                                     uint32_t *n_ids, void *ws, void *stream) {
    if (!pres || !tab || !n_ids || !ws || pc_span == 0 || pc_span > (1ull << 32))
        return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t nwords = (pc_span + 31) / 32;
    const uint64_t nblk = (nwords + DICT_WPB - 1) / DICT_WPB;
    uint32_t *bsum = (uint32_t *)ws;
    hipLaunchKernelGGL(dict_pass_a, dim3((unsigned)nblk), dim3(DICT_THREADS), 0, s, pres, pc_span,
                       nwords, tab, bsum);
    SYZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(dict_pass_b, dim3(1), dim3(1024), 0, s, bsum, nblk, n_ids);
    SYZ_LAUNCH_CHECK();
    hipLaunchKernelGGL(dict_pass_c, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0, s, tab,
                       nwords, bsum);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_dict_to_list_drop(const uint64_t *tab, uint64_t pc_span,
                                            uint32_t pc_lo, uint32_t drop, uint32_t *out,
                                            uint32_t *n_out, void *stream) {
    if (!tab || !out || !n_out || pc_span == 0) return SYZCOV_EINVAL;
    const uint64_t nwords = (pc_span + 31) / 32;
    hipLaunchKernelGGL(dict_to_list_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0,
                       (hipStream_t)stream, tab, nwords, pc_lo, drop, out, n_out);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_dict_to_list(const uint64_t *tab, uint64_t pc_span, uint32_t pc_lo,
                                       uint32_t *out, uint32_t *n_out, void *stream) {
    return syzcov_dev_dict_to_list_drop(tab, pc_span, pc_lo, SYZ_SENT, out, n_out, stream);
}

extern "C" int syzcov_dev_bytemap_op(int op, uint8_t *dst, const uint8_t *src, uint64_t nbytes,
                                     uint64_t *popcount_out, void *stream) {
    if (op < 0 || op > 3 || !dst || !src) return SYZCOV_EINVAL;
    if (((uintptr_t)dst | (uintptr_t)src) & 15) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long *pop = (unsigned long long *)popcount_out;
    if (pop) SYZ_HIP(hipMemsetAsync(pop, 0, sizeof(uint64_t), s));
    const uint64_t nvec = nbytes / 16;
    if (nvec) {
        hipLaunchKernelGGL(bytemap_op_kernel, dim3(grid_for(nvec, 256, 8192)), dim3(256), 0, s, op,
                           dst, src, nvec, pop);
        SYZ_LAUNCH_CHECK();
    }
    if (nbytes % 16) {
        hipLaunchKernelGGL(bytemap_tail_kernel, dim3(1), dim3(64), 0, s, op, dst, src, nvec * 16,
                           nbytes, pop);
        SYZ_LAUNCH_CHECK();
    }
    return 0;
}

namespace syz {
// A bitmap <-> a byte map (one byte per bit, 0 or 1): the shard bitmaps'
// uint8 MAX all-reduce of north_star (dist.py merge_bitmap_u8).  One thread
// per 32-bit word: 32 bytes written as two 16-byte stores, or read back.
__global__ __launch_bounds__(256) void bits_to_bytes_kernel(const uint32_t *__restrict__ bits,
                                                            uint64_t nwords,
                                                            uint8_t *__restrict__ bytes) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = bits[w];
        uint32_t q[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t n = (x >> (4 * j)) & 15u;  // bits 4j..4j+3 -> bytes 4j..4j+3
            q[j] = (n & 1u) | ((n & 2u) << 7) | ((n & 4u) << 14) | ((n & 8u) << 21);
        }
        uint4 *o = reinterpret_cast<uint4 *>(bytes + w * 32);
        o[0] = make_uint4(q[0], q[1], q[2], q[3]);
        o[1] = make_uint4(q[4], q[5], q[6], q[7]);
    }
}
__global__ __launch_bounds__(256) void bytes_to_bits_kernel(const uint8_t *__restrict__ bytes,
                                                            uint64_t nwords,
                                                            uint32_t *__restrict__ bits) {
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 *in = reinterpret_cast<const uint4 *>(bytes + w * 32);
        const uint4 a = in[0], b = in[1];
        const uint32_t q[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t v = q[j];
            const uint32_t n = ((v & 0xFFu) != 0) | (((v >> 8) & 0xFFu) != 0) << 1 |
                               (((v >> 16) & 0xFFu) != 0) << 2 | ((v >> 24) != 0) << 3;
            x |= n << (4 * j);
        }
        bits[w] = x;
    }
}
}  // namespace syz

extern "C" int syzcov_dev_bits_to_bytes(const uint32_t *bits, uint64_t nwords, uint8_t *bytes,
                                        void *stream) {
    if (!nwords) return 0;
    if (!bits || !bytes || ((uintptr_t)bytes & 15)) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(syz::bits_to_bytes_kernel, dim3(grid_for(nwords, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, bits, nwords, bytes);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_bytes_to_bits(const uint8_t *bytes, uint64_t nwords, uint32_t *bits,
                                        void *stream) {
    if (!nwords) return 0;
    if (!bits || !bytes || ((uintptr_t)bytes & 15)) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(syz::bytes_to_bits_kernel, dim3(grid_for(nwords, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, bytes, nwords, bits);
    SYZ_LAUNCH_CHECK();
    return 0;
}

namespace syz {
// Sorted PC list of a bitmap over [pc_lo, pc_lo + pc_span) (sentinel
// dropped, as a Union result would).  out == NULL: count only.
// pc_of_key (nullable): the bitmap is over dense keys (keys.hip); the list is
// mapped back to PCs (monotone, so it stays sorted).
int bitmap_to_list(const uint32_t *bm, uint64_t pc_span, uint32_t pc_lo, uint32_t *out,
                   size_t cap, int64_t *count, hipStream_t s, const uint32_t *pc_of_key) {
    const uint64_t nwords = (pc_span + 31) / 32;
    const uint64_t nblk = (nwords + DICT_WPB - 1) / DICT_WPB;
    void *buf = nullptr;
    const size_t o_bsum = align_up(nwords * 8, 256), o_n = o_bsum + align_up(nblk * 4, 256);
    if (hipMalloc(&buf, o_n + 256) != hipSuccess) return SYZCOV_ENOMEM;
    uint64_t *tab = (uint64_t *)buf;
    uint32_t *bsum = (uint32_t *)((uint8_t *)buf + o_bsum);
    uint32_t *dn = (uint32_t *)((uint8_t *)buf + o_n);
    int rc = 0;
    uint32_t hn = 0;
    uint32_t *dout = nullptr;
    do {
        hipLaunchKernelGGL(dict_pass_a_bits, dim3((unsigned)nblk), dim3(DICT_THREADS), 0, s, bm,
                           nwords, tab, bsum);
        hipLaunchKernelGGL(dict_pass_b, dim3(1), dim3(1024), 0, s, bsum, nblk, dn);
        hipLaunchKernelGGL(dict_pass_c, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0, s, tab,
                           nwords, bsum);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&hn, dn, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = SYZCOV_EHIP;
            break;
        }
        if (!out) {
            // count minus a present sentinel
            hipLaunchKernelGGL(dict_to_list_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0,
                               s, tab, nwords, pc_lo, SYZ_SENT, (uint32_t *)nullptr, dn);
        } else {
            if (hipMalloc(&dout, (size_t)hn * 4 + 4) != hipSuccess) {
                rc = SYZCOV_ENOMEM;
                break;
            }
            hipLaunchKernelGGL(dict_to_list_kernel, dim3(grid_for(nwords, 256, 16384)), dim3(256), 0,
                               s, tab, nwords, pc_lo, SYZ_SENT, dout, dn);
        }
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&hn, dn, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = SYZCOV_EHIP;
            break;
        }
        if (out) {
            if (hn > cap) {
                rc = SYZCOV_EINVAL;
                break;
            }
            if (pc_of_key && hn &&
                (rc = syzcov_dev_keys_to_pcs(pc_of_key, pc_span, dout, dout, nullptr, hn, s)))
                break;
            if (hn && (hipMemcpyAsync(out, dout, (size_t)hn * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                       hipStreamSynchronize(s) != hipSuccess)) {
                rc = SYZCOV_EHIP;
                break;
            }
        }
        *count = hn;
    } while (0);
    if (dout) hipFree(dout);
    hipFree(buf);
    return rc;
}
}  // namespace syz

namespace syz {
__global__ void minmax_kernel(const uint32_t *__restrict__ pcs, uint64_t n,
                              uint32_t *__restrict__ mm) {
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = pcs[i];
        lo = min(lo, v);
        hi = max(hi, v);
    }
    for (int d = 32; d >= 1; d >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor(lo, d, 64));
        hi = max(hi, (uint32_t)__shfl_xor(hi, d, 64));
    }
    if (__lane_id() == 0) {
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
    }
}

int minmax_pcs(const uint32_t *pcs, size_t n, uint32_t *mm, hipStream_t s) {
    const uint32_t init[2] = {0xFFFFFFFFu, 0u};
    SYZ_HIP(hipMemcpyAsync(mm, init, 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(minmax_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, pcs,
                       (uint64_t)n, mm);
    SYZ_LAUNCH_CHECK();
    return 0;
}
}  // namespace syz
