// prio.hip — prog.CalculatePriorities' dynamic part (prog/prio.go:137-154),
// normalizePrio (:158-192), the static combine (:29-38) and BuildChoiceTable
// (:202-228) on gfx950.
//
// Raw co-occurrence counts are the dense contraction D = AᵀA - diag(colsum A)
// over a prog x key matrix A, on i8 MFMA (v_mfma_i32_32x32x32_i8) with i32
// accumulation, so the counts are exact:
//   key mode 0 (reference-exact): the reference indexes prios by call
//     POSITION (prio.go:142-150 never reads Meta.ID), so A[p][k] = [k < len(p)];
//   key mode 1: A[p][c] = number of calls with syscall id c in program p.
// A is stored K-blocked: for each step of PK = 64 programs a contiguous
// [rows][64] byte block (key-major inside), so an MFMA fragment -- 16
// consecutive programs of one key -- is one 16-byte read, and one K step of
// every tile is one contiguous 80 KB region (L2-friendly; a plain key-major
// AT with a 1 MB row stride made the tiles' rows collide in the same L2 sets).  An all-ones key row at index C makes the GEMM also produce
// colsum(A) = D[i][C] for the diagonal correction.  Only tiles with I <= J are
// computed (D is symmetric) and mirrored; K (programs) is split across
// workgroups with exact int32 atomics in the epilogue.
//
// Counts convert to float32 as Go's repeated `+= 1.0` does: exact up to 2^24,
// then stuck at 2^24 (round-to-even), i.e. min(n, 16777216).  All float
// arithmetic uses explicit round-to-nearest intrinsics: no FMA contraction.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

namespace syz {

constexpr int PT = 128;  // output tile (keys) per workgroup
constexpr int PK = 64;   // programs per K-step

__host__ __device__ inline size_t prio_rows(int C) { return ((size_t)C + 1 + PT - 1) / PT * PT; }
__host__ __device__ inline size_t prio_ldp(size_t nprog) { return (nprog + PK - 1) / PK * PK; }
// byte offset of (key r, program p) in the K-blocked AT
__host__ __device__ inline size_t at_off(size_t r, size_t p, size_t rows) {
    return (p / PK) * (rows * PK) + r * PK + (p % PK);
}

// ---------------------------------------------------------------- A builders
// positional: AT[c][p] = (c < len[p]) for c < C, AT[ones][p] = (p < nprog)
// (ones = C for the full matrix; -1: no ones row, colsum computed apart).
// One workgroup per K block (64 programs, a contiguous rows x 64 B region):
// thread t owns program chunk t % 4 (its 16 lengths stay in registers) and
// rows t / 4 + 64 i, so a wave stores 1 KB contiguous per instruction.
__global__ __launch_bounds__(256) void prio_build_pos_kernel(const int32_t *__restrict__ lens,
                                                             size_t nprog, int C, int ones,
                                                             size_t rows, size_t ldp,
                                                             int8_t *__restrict__ at) {
    const size_t nkb = ldp / PK;
    const uint32_t t = threadIdx.x, ch = t & 3u;
    for (size_t kb = blockIdx.x; kb < nkb; kb += gridDim.x) {
        const size_t p0 = kb * PK + ch * 16;
        int32_t ln[16];
#pragma unroll
        for (int j = 0; j < 16; j++) ln[j] = p0 + j < nprog ? lens[p0 + j] : -1;  // -1: no program
        int8_t *blk = at + kb * (rows * PK) + ch * 16;
        for (size_t r = t >> 2; r < rows; r += 64) {
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t v = 0;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const int32_t L = ln[q * 4 + c];
                    const bool bit = (int)r < C ? (int32_t)r < L : ((int)r == ones && L >= 0);
                    v |= (uint32_t)bit << (8 * c);
                }
                w[q] = v;
            }
            *(uint4 *)(blk + r * PK) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

// by id: AT[cid][p] += 1 per call (byte counts in 32-bit atomics; <= 127
// per program is checked by the host wrapper's caller contract)
__global__ void prio_build_id_kernel(const uint64_t *__restrict__ prog_off,
                                     const uint16_t *__restrict__ ids, size_t nprog, int C,
                                     size_t rows, int8_t *__restrict__ at,
                                     uint32_t *__restrict__ err) {
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < nprog;
         p += (size_t)gridDim.x * blockDim.x) {
        for (uint64_t q = prog_off[p]; q < prog_off[p + 1]; q++) {
            const uint32_t c = ids[q];
            if ((int)c >= C) {
                *err = 1u;
                continue;
            }
            const size_t byte = at_off(c, p, rows);
            atomicAdd((unsigned int *)(at + (byte & ~(size_t)3)), 1u << (8 * (byte & 3)));
        }
        const size_t byte = at_off((size_t)C, p, rows);  // ones row
        atomicAdd((unsigned int *)(at + (byte & ~(size_t)3)), 1u << (8 * (byte & 3)));
    }
}

// ------------------------------------------------------------- MFMA AᵀA
// LDS image: [128 keys][64 programs] bytes, 16-B chunk index XOR-swizzled by
// (row >> 2) & 3 so a ds_read_b128 lane group hits distinct bank slots.
__device__ __forceinline__ uint32_t lds_off(uint32_t row, uint32_t chunk) {
    return row * PK + ((chunk ^ ((row >> 2) & 3u)) << 4);
}

// One K step (64 programs) of a wave's 64x64 sub-tile: 2 x 2 MFMA 32x32x32.
__device__ __forceinline__ void mfma_step(const int8_t *Asrc, const int8_t *Bsrc, uint32_t l,
                                          uint32_t wr, uint32_t wc, v16i (&acc)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
        const uint32_t ch = ks * 2 + (l >> 5);
        v4i fa[2], fb[2];
#pragma unroll
        for (int mi = 0; mi < 2; mi++)
            fa[mi] = *(const v4i *)(Asrc + lds_off(wr * 64 + mi * 32 + (l & 31), ch));
#pragma unroll
        for (int ni = 0; ni < 2; ni++)
            fb[ni] = *(const v4i *)(Bsrc + lds_off(wc * 64 + ni * 32 + (l & 31), ch));
#pragma unroll
        for (int mi = 0; mi < 2; mi++)
#pragma unroll
            for (int ni = 0; ni < 2; ni++)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
    }
}

// Workgroup -> (tile, K split).  Splits are grouped by XCD: consecutive
// workgroup ids go to the 8 XCDs round-robin, so workgroup b runs on XCD
// b % 8 and the `gpx` K splits of an XCD run there with ALL their tiles at
// the same time.  The tiles of one split stream the same A rows over the same
// K range, so each operand chunk comes from HBM once per XCD and is re-read
// by the other tiles from that XCD's L2 (K splits spread over XCDs instead
// made every XCD fetch every chunk).
// GEN (positional, active keys): no AT at all -- each thread builds its
// 16-byte operand chunks in registers from the 16 program lengths of the
// chunk (byte j of key row r = [r < len(p_j)], the ones row = [p_j exists]),
// so the only HBM stream is the lengths (4 B per program).
__device__ __forceinline__ uint4 gen_chunk(const int32_t (&L)[16], int r, int ones) {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t v = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const int32_t len = L[q * 4 + c];
            v |= (uint32_t)(r == ones ? len >= 0 : r < len) << (8 * c);
        }
        w[q] = v;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool GEN>
__global__ __launch_bounds__(256) void prio_gemm_kernel(const int8_t *__restrict__ at, size_t ldp,
                                                        size_t kchunk, int ntile_dim,
                                                        int ntiles, int gpx,
                                                        int32_t *__restrict__ counts,
                                                        size_t rows, size_t ldc,
                                                        int32_t *__restrict__ part,
                                                        const int32_t *__restrict__ lens,
                                                        size_t nprog, int ones) {
    __shared__ __attribute__((aligned(16))) int8_t As[2][PT * PK];
    __shared__ __attribute__((aligned(16))) int8_t Bs[2][PT * PK];
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    const int tile = (int)(slot % (uint32_t)ntiles);
    const size_t split = (size_t)xcd * gpx + slot / (uint32_t)ntiles;
    // tile -> (I, J) with I <= J, row-major over the upper triangle
    int I = 0, rem = tile;
    while (rem >= ntile_dim - I) {
        rem -= ntile_dim - I;
        I++;
    }
    const int J = I + rem;
    const bool diag = I == J;
    const size_t i0 = (size_t)I * PT, j0 = (size_t)J * PT;
    const size_t kb0 = split * kchunk, kb1 = std::min(kb0 + kchunk, ldp);
    const uint32_t t = threadIdx.x, l = __lane_id(), w = t >> 6;
    const uint32_t wr = w >> 1, wc = w & 1;
    v16i acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0;

    // software pipeline, two K steps deep: step i+2's operands are loaded
    // into registers (set i % 2, just stored to LDS) while step i's MFMAs
    // run, so a load has two compute phases to arrive; two LDS buffers, one
    // barrier per step.  The loop is unrolled by two with named register sets
    // (arrays indexed by the set went to scratch).
    const uint32_t row0 = t >> 2, row1 = (t + 256u) >> 2, chq = t & 3u;  // chunk of both rows
    const uint32_t lo0 = lds_off(row0, chq), lo1 = lds_off(row1, chq);
    auto ld = [&](size_t kb, uint32_t base, uint32_t row) -> uint4 {
        return *(const uint4 *)(at + (kb / PK) * (rows * PK) + chq * 16 + (base + row) * PK);
    };
    uint4 a00, a01, b00, b01, a10, a11, b10, b11;
#define PRIO_LOAD(SET, KB)                                   \
    do {                                                     \
        a##SET##0 = ld((KB), (uint32_t)i0, row0);            \
        a##SET##1 = ld((KB), (uint32_t)i0, row1);            \
        if (!diag) {                                         \
            b##SET##0 = ld((KB), (uint32_t)j0, row0);        \
            b##SET##1 = ld((KB), (uint32_t)j0, row1);        \
        }                                                    \
    } while (0)
#define PRIO_STEP(SET, KB)                                                          \
    do {                                                                            \
        *(uint4 *)(As[SET] + lo0) = a##SET##0;                                      \
        *(uint4 *)(As[SET] + lo1) = a##SET##1;                                      \
        if (!diag) {                                                                \
            *(uint4 *)(Bs[SET] + lo0) = b##SET##0;                                  \
            *(uint4 *)(Bs[SET] + lo1) = b##SET##1;                                  \
        }                                                                           \
        __syncthreads();                                                            \
        if ((KB) + 2 * PK < kb1) PRIO_LOAD(SET, (KB) + 2 * PK);                     \
        mfma_step(As[SET], diag ? As[SET] : Bs[SET], l, wr, wc, acc);               \
    } while (0)
    // GEN: the 16 lengths of this thread's program chunk (-1: no program)
    int32_t L0[16], L1[16];
    auto load16 = [&](size_t kb, int32_t (&L)[16]) {
        const size_t p0 = kb + chq * 16;
        if (p0 + 16 <= nprog) {
            const int4 *src = reinterpret_cast<const int4 *>(lens + p0);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int4 v = src[q];
                L[q * 4] = v.x;
                L[q * 4 + 1] = v.y;
                L[q * 4 + 2] = v.z;
                L[q * 4 + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) L[j] = p0 + j < nprog ? lens[p0 + j] : -1;
        }
    };
#define GEN_STEP(SET, KB)                                                           \
    do {                                                                            \
        *(uint4 *)(As[SET] + lo0) = gen_chunk(L##SET, (int)(i0 + row0), ones);      \
        *(uint4 *)(As[SET] + lo1) = gen_chunk(L##SET, (int)(i0 + row1), ones);      \
        if (!diag) {                                                                \
            *(uint4 *)(Bs[SET] + lo0) = gen_chunk(L##SET, (int)(j0 + row0), ones);  \
            *(uint4 *)(Bs[SET] + lo1) = gen_chunk(L##SET, (int)(j0 + row1), ones);  \
        }                                                                           \
        __syncthreads();                                                            \
        if ((KB) + 2 * PK < kb1) load16((KB) + 2 * PK, L##SET);                     \
        mfma_step(As[SET], diag ? As[SET] : Bs[SET], l, wr, wc, acc);               \
    } while (0)
    if (GEN) {
        if (kb0 < kb1) load16(kb0, L0);
        if (kb0 + PK < kb1) load16(kb0 + PK, L1);
        for (size_t kb = kb0; kb < kb1; kb += 2 * PK) {
            GEN_STEP(0, kb);
            if (kb + PK < kb1) GEN_STEP(1, kb + PK);
        }
    } else {
        if (kb0 < kb1) PRIO_LOAD(0, kb0);
        if (kb0 + PK < kb1) PRIO_LOAD(1, kb0 + PK);
        for (size_t kb = kb0; kb < kb1; kb += 2 * PK) {
            PRIO_STEP(0, kb);
            if (kb + PK < kb1) PRIO_STEP(1, kb + PK);
        }
    }
#undef GEN_STEP
#undef PRIO_STEP
#undef PRIO_LOAD
    // epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    int32_t *pt = part ? part + (split * (size_t)ntiles + tile) * (PT * PT) : nullptr;
#pragma unroll
    for (int mi = 0; mi < 2; mi++)
#pragma unroll
        for (int ni = 0; ni < 2; ni++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int32_t v = acc[mi][ni][r];
                const uint32_t lr = wr * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
                const uint32_t lc = wc * 64 + ni * 32 + (l & 31);
                if (pt) {  // few tiles, many K splits: plain partial-tile stores
                    pt[lr * PT + lc] = v;
                    continue;
                }
                if (!v) continue;
                const size_t row = i0 + lr, col = j0 + lc;
                atomicAdd(&counts[row * ldc + col], v);
                if (!diag) atomicAdd(&counts[col * ldc + row], v);
            }
}

// Dense mode, 256 x 256 tiles (rows a multiple of 256): the 128 x 128 tile
// above reads 2 KB of LDS per 32x32x32 MFMA pair and writes 16 KB per K step
// for 8 MFMAs per wave, so its LDS traffic (384 cycles per step) exceeds its
// MFMA time (256 cycles per SIMD): LDS-bound at 0.30 of the i8 peak.  Here
// 8 waves (two per SIMD) each own a 64 x 128 sub-tile (2 x 4 MFMA 32x32x32,
// 128 accumulators): per K step a SIMD's two waves issue 32 MFMAs (1024
// cycles) against 96 KB of fragment reads and 32 KB of staging writes per CU
// (1024 cycles of LDS), with the second wave hiding the first's waits.  (One
// wave per SIMD with a 128 x 128 sub-tile: the 256 accumulators made the
// compiler shuttle them between AGPRs and VGPRs, ~1000 moves per K loop.)
// One workgroup per CU, every tile an equal share of K (diagonal tiles too),
// so the grid of tiles x splits runs in one round; partial tiles go to `part`
// and prio_reduce_kernel<256> sums the splits.
constexpr int PT2 = 256;
constexpr int G2_THREADS = 512;
__device__ __forceinline__ void mfma_step256(const int8_t *Asrc, const int8_t *Bsrc, uint32_t l,
                                             uint32_t wr, uint32_t wc, v16i (&acc)[2][4]) {
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
        const uint32_t ch = ks * 2 + (l >> 5);
        v4i fa[2], fb[4];
#pragma unroll
        for (int mi = 0; mi < 2; mi++)
            fa[mi] = *(const v4i *)(Asrc + lds_off(wr * 64 + mi * 32 + (l & 31), ch));
#pragma unroll
        for (int ni = 0; ni < 4; ni++)
            fb[ni] = *(const v4i *)(Bsrc + lds_off(wc * 128 + ni * 32 + (l & 31), ch));
#pragma unroll
        for (int mi = 0; mi < 2; mi++)
#pragma unroll
            for (int ni = 0; ni < 4; ni++)
                acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
    }
}

// Operands go global -> LDS directly (global_load_lds, 16 bytes a lane): a
// wave-instruction writes 1 KB = 16 rows x 64 programs contiguously, so the
// XOR swizzle of lds_off is applied to each lane's SOURCE chunk.  G2_NS stages
// of 32 KB (A rows, then B rows) in one dynamic LDS block; step k + G2_NS - 1
// is issued right after step k's barrier, and the wait before a barrier is a
// counted vmcnt (the later steps' loads stay in flight across it) with a raw
// s_barrier (__syncthreads would drain vmcnt to 0).  (Register staging, two
// sets in flight: 1.22 ms for the C4 contraction, load latency exposed.)
constexpr int G2_NS = 4;
constexpr size_t G2_STAGE = 2 * PT2 * PK;
constexpr size_t G2_LDS = G2_NS * G2_STAGE;  // 128 KB
__device__ __forceinline__ void g2_glds(const int8_t *src, int8_t *dst) {
    __builtin_amdgcn_global_load_lds((const void *)src,
                                     (__attribute__((address_space(3))) void *)dst, 16, 0, 0);
}

__global__ __launch_bounds__(G2_THREADS, 1) void prio_gemm256_kernel(const int8_t *__restrict__ at,
                                                                     size_t ldp, size_t kchunk,
                                                                     int ntile_dim, int ntiles,
                                                                     int gpx, size_t rows,
                                                                     int32_t *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) int8_t g2_lds[];
    // splits grouped by XCD (prio_gemm_kernel): an XCD's splits run with all
    // their tiles, so each K block of AT comes from HBM once per XCD
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    const int tile = (int)(slot % (uint32_t)ntiles);
    const size_t split = (size_t)xcd * gpx + slot / (uint32_t)ntiles;
    int I = 0, rem = tile;
    while (rem >= ntile_dim - I) {
        rem -= ntile_dim - I;
        I++;
    }
    const int J = I + rem;
    const bool diag = I == J;
    const size_t i0 = (size_t)I * PT2, j0 = (size_t)J * PT2;
    const size_t kb0 = std::min(split * kchunk, ldp), kb1 = std::min(kb0 + kchunk, ldp);
    const uint32_t nsteps = (uint32_t)((kb1 - kb0) / PK);
    const uint32_t t = threadIdx.x, l = __lane_id(), w = wave_readfirstlane(t >> 6);
    const uint32_t wr = w >> 1, wc = w & 1;
    v16i acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0;
    // wave w stages rows 32 w .. 32 w + 31 of A (and of B): two 16-row blocks;
    // lane l of block q lands at row 32 w + 16 q + l / 4, slot l & 3, which
    // holds chunk (l & 3) ^ ((row >> 2) & 3)
    const uint32_t r0 = 32 * w + (l >> 2), r1 = r0 + 16;
    const size_t sa0 = (i0 + r0) * PK + (((l & 3u) ^ ((r0 >> 2) & 3u)) << 4);
    const size_t sa1 = (i0 + r1) * PK + (((l & 3u) ^ ((r1 >> 2) & 3u)) << 4);
    const size_t sb0 = (j0 + r0) * PK + (((l & 3u) ^ ((r0 >> 2) & 3u)) << 4);
    const size_t sb1 = (j0 + r1) * PK + (((l & 3u) ^ ((r1 >> 2) & 3u)) << 4);
    const uint32_t d0 = 32 * w * PK, d1 = d0 + 16 * PK;
    auto issue = [&](uint32_t k) {
        const int8_t *src = at + (kb0 / PK + k) * (rows * PK);
        int8_t *st = g2_lds + (k % G2_NS) * G2_STAGE;
        g2_glds(src + sa0, st + d0);
        g2_glds(src + sa1, st + d1);
        if (!diag) {
            g2_glds(src + sb0, st + PT2 * PK + d0);
            g2_glds(src + sb1, st + PT2 * PK + d1);
        }
    };
    for (uint32_t k = 0; k < (uint32_t)G2_NS - 1 && k < nsteps; k++) issue(k);
    for (uint32_t k = 0; k < nsteps; k++) {
        // this wave's loads of step k are done once at most the later steps'
        // (2 or 4 a step) are outstanding
        const uint32_t ahead = min((uint32_t)G2_NS - 2, nsteps - 1 - k);
        if (diag) {
            if (ahead >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        // (stage (k + NS - 1) % NS was read in step k - 1, before the barrier)
        if (k + G2_NS - 1 < nsteps) issue(k + G2_NS - 1);
        const int8_t *st = g2_lds + (k % G2_NS) * G2_STAGE;
        mfma_step256(st, diag ? st : st + PT2 * PK, l, wr, wc, acc);
    }
    // epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    int32_t *pt = part + (split * (size_t)ntiles + tile) * (PT2 * PT2);
#pragma unroll
    for (int mi = 0; mi < 2; mi++)
#pragma unroll
        for (int ni = 0; ni < 4; ni++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const uint32_t lr = wr * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
                const uint32_t lc = wc * 128 + ni * 32 + (l & 31);
                pt[lr * PT2 + lc] = acc[mi][ni][r];
            }
}

// counts (ldc stride, zeroed) += the partial tiles of the K splits, mirrored
// below the diagonal.  blockIdx.y takes every gridDim.y-th split, so each
// count gets gridDim.y atomic adds (coalesced loads, 8 splits in flight per
// thread) instead of one thread summing all splits in a latency chain.
// The ones row (index `ones`, >= every nonzero key) yields colsum in its
// column: it goes to column C, the slot prio_finish reads it from.
template <int TT = PT>
__global__ __launch_bounds__(256) void prio_reduce_kernel(const int32_t *__restrict__ part,
                                                          size_t splits, int ntiles, int ntile_dim,
                                                          int32_t *__restrict__ counts,
                                                          size_t ldc, int ones, int C) {
    const size_t per = (size_t)ntiles * TT * TT;
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= per) return;
    int32_t sum = 0;
    size_t sp = blockIdx.y;
    for (; sp + 7 * gridDim.y < splits; sp += 8 * gridDim.y) {
        int32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = part[(sp + u * gridDim.y) * per + e];
#pragma unroll
        for (int u = 0; u < 8; u++) sum += v[u];
    }
    for (; sp < splits; sp += gridDim.y) sum += part[sp * per + e];
    if (!sum) return;
    const int tile = (int)(e / (TT * TT));
    const uint32_t lr = (uint32_t)(e % (TT * TT)) / TT, lc = (uint32_t)(e % TT);
    int I = 0, rem = tile;
    while (rem >= ntile_dim - I) {
        rem -= ntile_dim - I;
        I++;
    }
    const size_t row = (size_t)I * TT + lr, col = (size_t)(I + rem) * TT + lc;
    // the ones row lies in the last row block, so every key meets it once as
    // a COLUMN (tiles (I, last) and the diagonal last tile); its row copy in
    // the diagonal tile is the same numbers and is skipped
    if ((int)row == ones) return;
    // one writer per count when every split is summed here (gridDim.y == 1):
    // a plain read-add-write, else atomics
    auto add = [&](size_t x) {
        if (gridDim.y == 1) counts[x] += sum; else atomicAdd(&counts[x], sum);
    };
    if ((int)col == ones) {
        if ((int)row < C) add(row * ldc + C);
        return;
    }
    add(row * ldc + col);
    if (rem) add(col * ldc + row);
}

// Positional colsum: counts[i][C] = #{p : len(p) > i} (the diagonal
// correction), from a length histogram and a suffix sum.
__global__ __launch_bounds__(256) void prio_len_hist_kernel(const int32_t *__restrict__ lens,
                                                            size_t nprog, int C,
                                                            uint32_t *__restrict__ hist) {
    extern __shared__ uint32_t h[];
    for (int i = threadIdx.x; i <= C; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < nprog;
         p += (size_t)gridDim.x * blockDim.x) {
        const int32_t L = lens[p];
        atomicAdd(&h[L < 0 ? 0 : (L > C ? C : L)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= C; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

__global__ __launch_bounds__(1024) void prio_colsum_kernel(const uint32_t *__restrict__ hist,
                                                           int C, int32_t *__restrict__ counts,
                                                           size_t ldc) {
    // colsum[i] = sum_{L > i} hist[L]: suffix sum in LDS, then parallel stores
    extern __shared__ int32_t sfx[];
    for (int i = threadIdx.x; i <= C; i += blockDim.x) sfx[i] = (int32_t)hist[i];
    __syncthreads();
    if (threadIdx.x == 0)
        for (int i = C - 1; i >= 0; i--) sfx[i] += sfx[i + 1];
    __syncthreads();
    for (int i = threadIdx.x; i < C; i += blockDim.x) counts[(size_t)i * ldc + C] = sfx[i + 1];
}

// ---------------------------------------------------- finish: float + normalize
// counts -> float32 per Go's `+= 1.0` accumulation, diagonal corrected,
// then normalizePrio per row, then * static.  One workgroup per row.
__device__ __forceinline__ float go_f32_count(int64_t n) {
    return n >= 16777216 ? 16777216.0f : (float)n;
}

template <int THREADS>
__device__ __forceinline__ void row_stats(const float *__restrict__ row, int C, float *mx,
                                          float *mn, int *nz, float *red) {
    float lmax = 0.0f, lmin = 1e10f;
    int lz = 0;
    for (int i = threadIdx.x; i < C; i += THREADS) {
        const float p = row[i];
        lmax = fmaxf(lmax, p);
        if (p != 0.0f) lmin = fminf(lmin, p);
        lz += p == 0.0f;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        lmax = fmaxf(lmax, __shfl_xor(lmax, d, 64));
        lmin = fminf(lmin, __shfl_xor(lmin, d, 64));
        lz += __shfl_xor(lz, d, 64);
    }
    const int w = threadIdx.x >> 6;
    if (__lane_id() == 0) {
        red[w] = lmax;
        red[THREADS / 64 + w] = lmin;
        ((int *)red)[2 * THREADS / 64 + w] = lz;
    }
    __syncthreads();
    float m0 = 0.0f, m1 = 1e10f;
    int z = 0;
    for (int q = 0; q < THREADS / 64; q++) {
        m0 = fmaxf(m0, red[q]);
        m1 = fminf(m1, red[THREADS / 64 + q]);
        z += ((int *)red)[2 * THREADS / 64 + q];
    }
    __syncthreads();
    *mx = m0;
    *mn = m1;
    *nz = z;
}

// prio.go:158-192 on one row (row in LDS or global), exact float32.
template <int THREADS>
__device__ __forceinline__ void normalize_row(float *__restrict__ row, int C, float *red) {
    float mx, mn;
    int nz;
    row_stats<THREADS>(row, C, &mx, &mn, &nz, red);
    if (nz != 0) mn = __fdiv_rn(mn, __fmul_rn(2.0f, (float)nz));
    const float den = __fsub_rn(mx, mn);
    for (int i = threadIdx.x; i < C; i += THREADS) {
        float p = row[i];
        if (mx == 0.0f) {
            row[i] = 1.0f;
            continue;
        }
        if (p == 0.0f) p = mn;
        p = __fadd_rn(__fmul_rn(__fdiv_rn(__fsub_rn(p, mn), den), 0.9f), 0.1f);
        if (p > 1.0f) p = 1.0f;
        row[i] = p;
    }
    __syncthreads();
}

constexpr int FIN_THREADS = 256;

__global__ __launch_bounds__(FIN_THREADS) void prio_finish_kernel(
    const int32_t *__restrict__ counts, size_t rows, int C, const float *__restrict__ st,
    float *__restrict__ out, uint32_t *__restrict__ raw) {
    extern __shared__ float rowbuf[];
    __shared__ float red[3 * FIN_THREADS / 64];
    const int i = blockIdx.x;
    const int32_t *crow = counts + (size_t)i * rows;
    const int64_t colsum = crow[C];
    for (int j = threadIdx.x; j < C; j += FIN_THREADS) {
        int64_t n = crow[j];
        if (j == i) n -= colsum;  // D = AᵀA - diag(colsum A)
        if (raw) raw[(size_t)i * C + j] = (uint32_t)n;
        rowbuf[j] = go_f32_count(n);
    }
    __syncthreads();
    normalize_row<FIN_THREADS>(rowbuf, C, red);
    for (int j = threadIdx.x; j < C; j += FIN_THREADS) {
        float p = rowbuf[j];
        if (st) p = __fmul_rn(p, st[(size_t)i * C + j]);  // prio.go:34 dynamic[i][j] *= p
        out[(size_t)i * C + j] = p;
    }
}

__global__ __launch_bounds__(FIN_THREADS) void prio_normalize_kernel(float *__restrict__ prios,
                                                                     int C) {
    __shared__ float red[3 * FIN_THREADS / 64];
    normalize_row<FIN_THREADS>(prios + (size_t)blockIdx.x * C, C, red);
}

// prio.go:202-228: run[i][j] = sum_{j' <= j, enabled[j']} int(prios[i][j'] * 1000)
__global__ __launch_bounds__(FIN_THREADS) void choice_table_kernel(
    const float *__restrict__ prios, const uint8_t *__restrict__ enabled, int C,
    int64_t *__restrict__ run) {
    __shared__ int64_t wsum[FIN_THREADS / 64 + 1];
    const int i = blockIdx.x;
    if (enabled && !enabled[i]) return;  // nil row
    int64_t carry = 0;
    for (int c0 = 0; c0 < C; c0 += FIN_THREADS) {
        const int j = c0 + threadIdx.x;
        int64_t v = 0;
        if (j < C && (!enabled || enabled[j]))
            v = (int64_t)__fmul_rn(prios[(size_t)i * C + j], 1000.0f);  // truncation, as Go int()
        // block inclusive scan (int64)
        int64_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
            int64_t y = __shfl_up(x, d, 64);
            if ((int)__lane_id() >= d) x += y;
        }
        const int w = threadIdx.x >> 6;
        if (__lane_id() == 63) wsum[w] = x;
        __syncthreads();
        int64_t pre = 0;
        for (int q = 0; q < w; q++) pre += wsum[q];
        int64_t tot = 0;
        for (int q = 0; q < FIN_THREADS / 64; q++) tot += wsum[q];
        if (j < C) run[(size_t)i * C + j] = carry + pre + x;
        carry += tot;
        __syncthreads();
    }
}

// calcStaticPriorities (prio.go:40-135) from the usage table: one workgroup
// per row c0 accumulates prios[c0][c1] += w0 * w1 over the usage ids holding
// c0 in ascending id order (one fixed order of Go's map walk; the members of
// one id are distinct calls, so a row update per id is race-free), sets the
// diagonal to the row max (:124-132) and normalises the row (:133).
__global__ __launch_bounds__(FIN_THREADS) void static_prio_kernel(
    const uint32_t *__restrict__ id_off, const uint16_t *__restrict__ id_calls,
    const float *__restrict__ id_w, const uint32_t *__restrict__ call_off,
    const uint32_t *__restrict__ call_ids, const float *__restrict__ call_w, int C,
    float *__restrict__ out) {
    extern __shared__ float row[];
    __shared__ float red[3 * FIN_THREADS / 64];
    const int c0 = blockIdx.x;
    for (int j = threadIdx.x; j < C; j += FIN_THREADS) row[j] = 0.0f;
    __syncthreads();
    for (uint32_t q = call_off[c0]; q < call_off[c0 + 1]; q++) {
        const uint32_t id = call_ids[q];
        const float w0 = call_w[q];
        for (uint32_t m = id_off[id] + threadIdx.x; m < id_off[id + 1]; m += FIN_THREADS) {
            const int c1 = id_calls[m];
            if (c1 != c0) row[c1] = __fadd_rn(row[c1], __fmul_rn(w0, id_w[m]));
        }
        __syncthreads();
    }
    // diagonal = row max (the diagonal itself is still 0 here)
    float mx = 0.0f, mn;
    int nz;
    row_stats<FIN_THREADS>(row, C, &mx, &mn, &nz, red);
    if (threadIdx.x == 0) row[c0] = mx;
    __syncthreads();
    normalize_row<FIN_THREADS>(row, C, red);
    for (int j = threadIdx.x; j < C; j += FIN_THREADS) out[(size_t)c0 * C + j] = row[j];
}


// ChoiceTable.Choose (prio.go:230-249) for a batch of (call, x) draws, where
// x is the caller's r.Intn(run[last]) (Go's math/rand stays with the caller):
// i = sort.SearchInts(run[call], x), the first i with run[i] >= x.
//   out = i   the call is enabled (Choose returns i)
//   out = -1  rejected: Choose draws again (`continue`)
//   out = -2  call < 0 or a nil (disabled) row: Choose picks uniformly from
//             enabledCalls
// An x outside [0, run[call][C-1]) (r.Intn's range) sets *err.
__global__ void choose_kernel(const int64_t *__restrict__ run, const uint8_t *__restrict__ enabled,
                              int C, const int32_t *__restrict__ calls,
                              const int64_t *__restrict__ x, uint64_t nq, int32_t *__restrict__ out,
                              uint32_t *__restrict__ err) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nq;
         k += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t c = calls[k];
        if (c >= C) {
            *err = 1u;
            out[k] = -3;
            continue;
        }
        if (c < 0 || (enabled && !enabled[c])) {
            out[k] = -2;
            continue;
        }
        const int64_t *row = run + (uint64_t)c * C;
        const int64_t xx = x[k];
        if (xx < 0 || xx >= row[C - 1]) {
            *err = 1u;
            out[k] = -3;
            continue;
        }
        int lo = 0, hi = C - 1;  // row[C-1] > xx, so the answer is < C
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (row[mid] >= xx) hi = mid; else lo = mid + 1;
        }
        out[k] = (!enabled || enabled[lo]) ? lo : -1;
    }
}

}  // namespace syz

using namespace syz;

extern "C" int syzcov_dev_static_prio(const uint32_t *id_off, const uint16_t *id_calls,
                                      const float *id_w, const uint32_t *call_off,
                                      const uint32_t *call_ids, const float *call_w, int C,
                                      float *out, void *stream) {
    if (C <= 0 || !id_off || !id_calls || !id_w || !call_off || !call_ids || !call_w || !out)
        return SYZCOV_EINVAL;
    hipLaunchKernelGGL(static_prio_kernel, dim3(C), dim3(FIN_THREADS), C * sizeof(float),
                       (hipStream_t)stream, id_off, id_calls, id_w, call_off, call_ids, call_w, C,
                       out);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" size_t syzcov_dev_prio_rows(int C) { return prio_rows(C); }
extern "C" size_t syzcov_dev_prio_ldp(size_t nprog) { return prio_ldp(nprog); }

extern "C" int syzcov_dev_prio_build_at(int key_mode, const int32_t *lens,
                                        const uint64_t *prog_off, const uint16_t *call_ids,
                                        size_t nprog, int C, int8_t *at, size_t ldp,
                                        uint32_t *err_flag, void *stream) {
    if (C <= 0 || !at || ldp % PK || ldp < nprog) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const size_t rows = prio_rows(C);
    if (key_mode == 0) {
        if (nprog && !lens) return SYZCOV_EINVAL;
        hipLaunchKernelGGL(prio_build_pos_kernel, dim3(grid_for(ldp / PK, 1, 16384)), dim3(256), 0,
                           s, lens, nprog, C, C, rows, ldp, at);
        SYZ_LAUNCH_CHECK();
        return 0;
    }
    if (key_mode != 1 || (nprog && (!prog_off || !call_ids || !err_flag))) return SYZCOV_EINVAL;
    SYZ_HIP(hipMemsetAsync(at, 0, rows * ldp, s));
    if (nprog) {
        hipLaunchKernelGGL(prio_build_id_kernel, dim3(grid_for(nprog, 256, 8192)), dim3(256), 0, s,
                           prog_off, call_ids, nprog, C, rows, at, err_flag);
        SYZ_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" int syzcov_dev_prio_counts(const int8_t *at, size_t ldp, size_t nprog, int C,
                                      int32_t *counts, void *stream) {
    if (C <= 0 || !at || !counts || ldp % PK || ldp < nprog) return SYZCOV_EINVAL;
    if (nprog == 0) return 0;
    const size_t rows = prio_rows(C);
    const int nt = (int)(rows / PT);
    const int ntiles = nt * (nt + 1) / 2;
    // K splits: a multiple of the 8 XCDs, gpx per XCD, enough workgroups to
    // fill the chip ~3x over.  Splits past the end of K have empty ranges.
    const size_t nk = ldp / PK;
    int gpx = (int)std::max<size_t>(1, std::min<size_t>((nk + 7) / 8,
                                                              (768 / 8 + ntiles - 1) / ntiles));
    const size_t splits = 8 * (size_t)gpx;
    const size_t kchunk = (nk + splits - 1) / splits * PK;
    hipLaunchKernelGGL(prio_gemm_kernel<false>, dim3((unsigned)(ntiles * splits)), dim3(256), 0,
                       (hipStream_t)stream, at, ldp, kchunk, nt, ntiles, gpx, counts, rows, rows,
                       (int32_t *)nullptr, (const int32_t *)nullptr, (size_t)0, -1);
    SYZ_LAUNCH_CHECK();
    return 0;
}

// Dense mode on 256 x 256 tiles (prio_gemm256_kernel): one workgroup per CU,
// 8 * gpx K splits grouped by XCD, partial tiles in ws, one reduction.
static bool g256_plan(size_t nprog, int C, int *nt, int *ntiles, int *gpx, size_t *kchunk) {
    const size_t rows = prio_rows(C);
    if (rows % PT2) return false;
    *nt = (int)(rows / PT2);
    *ntiles = *nt * (*nt + 1) / 2;
    int cus = 256, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const size_t nk = prio_ldp(nprog) / PK;
    // the most splits (a multiple of the 8 XCDs) with tiles x splits <= CUs
    *gpx = std::max(1, cus / (8 * *ntiles));
    *gpx = (int)std::min<size_t>(*gpx, (nk + 7) / 8);
    const size_t splits = 8 * (size_t)*gpx;
    *kchunk = (nk + splits - 1) / splits * PK;
    return true;
}

extern "C" size_t syzcov_dev_prio_counts_ws_size(size_t nprog, int C) {
    int nt, ntiles, gpx;
    size_t kc;
    if (C <= 0 || nprog == 0 || !g256_plan(nprog, C, &nt, &ntiles, &gpx, &kc)) return 0;
    return align_up(8 * (size_t)gpx * ntiles * PT2 * PT2 * 4, 256);
}

extern "C" int syzcov_dev_prio_counts_ws(const int8_t *at, size_t ldp, size_t nprog, int C,
                                         int32_t *counts, void *ws, size_t ws_size, void *stream) {
    if (C <= 0 || !at || !counts || ldp % PK || ldp < nprog) return SYZCOV_EINVAL;
    if (nprog == 0) return 0;
    const size_t need = syzcov_dev_prio_counts_ws_size(nprog, C);
    if (!need || !ws || ws_size < need)  // no 256-row tiling (or no workspace): 128 x 128 tiles
        return syzcov_dev_prio_counts(at, ldp, nprog, C, counts, stream);
    int nt, ntiles, gpx;
    size_t kc;
    g256_plan(nprog, C, &nt, &ntiles, &gpx, &kc);
    const size_t rows = prio_rows(C), splits = 8 * (size_t)gpx;
    hipStream_t s = (hipStream_t)stream;
    static std::atomic<uint32_t> g2_attr{0};
    if (int rc = set_dyn_lds_once((const void *)prio_gemm256_kernel, (uint32_t)G2_LDS, g2_attr))
        return rc;
    hipLaunchKernelGGL(prio_gemm256_kernel, dim3((unsigned)(ntiles * splits)), dim3(G2_THREADS), G2_LDS, s, at,
                       ldp, kc, nt, ntiles, gpx, rows, (int32_t *)ws);
    // the ones row (index C) yields colsum in column C, as prio_gemm_kernel's
    // atomics leave it
    hipLaunchKernelGGL(prio_reduce_kernel<PT2>,
                       dim3((unsigned)(((size_t)ntiles * PT2 * PT2 + 255) / 256), 1), dim3(256), 0,
                       s, (const int32_t *)ws, splits, ntiles, nt, counts, rows, C, C);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_prio_finish(const int32_t *counts, int C, const float *static_prios,
                                      float *out, uint32_t *raw_out, void *stream) {
    if (C <= 0 || !counts || !out) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(prio_finish_kernel, dim3(C), dim3(FIN_THREADS), C * sizeof(float),
                       (hipStream_t)stream, counts, prio_rows(C), C, static_prios, out, raw_out);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_normalize_prio(float *prios, int C, void *stream) {
    if (C <= 0 || !prios) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(prio_normalize_kernel, dim3(C), dim3(FIN_THREADS), 0, (hipStream_t)stream,
                       prios, C);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_choice_table(const float *prios, const uint8_t *enabled, int C,
                                       int64_t *run, void *stream) {
    if (C <= 0 || !prios || !run) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(choice_table_kernel, dim3(C), dim3(FIN_THREADS), 0, (hipStream_t)stream,
                       prios, enabled, C, run);
    SYZ_LAUNCH_CHECK();
    return 0;
}

extern "C" int syzcov_dev_choose(const int64_t *run, const uint8_t *enabled, int C,
                                 const int32_t *calls, const int64_t *x, size_t nq, int32_t *out,
                                 uint32_t *err_flag, void *stream) {
    if (nq == 0) return 0;
    if (C <= 0 || !run || !calls || !x || !out || !err_flag) return SYZCOV_EINVAL;
    hipLaunchKernelGGL(choose_kernel, dim3(grid_for(nq, 256, 8192)), dim3(256), 0,
                       (hipStream_t)stream, run, enabled, C, calls, x, (uint64_t)nq, out, err_flag);
    SYZ_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------- positional, active rows
// The reference's positional counts are zero for every key k >= max len
// (A[p][k] = [k < len(p)]), so the contraction runs over the first
// rows_act = roundup(max_len + 1, 128) keys only, with the ones row (colsum)
// at index max_len.  The operands are generated in registers from the
// program lengths (no AT in HBM); K is split over many workgroups whose
// partial tiles a reduction sums (a handful of tiles: atomics would put
// hundreds of adds on every count).  C4 (max len 120): one 128 x 128 tile,
// 4 MB of lengths read, instead of 55 tiles over a 1.28 GB AT.
static void pos_plan(size_t nprog, int C, int max_len, size_t *rows_act, size_t *ntiles,
                     size_t *splits, size_t *kchunk) {
    const size_t ra = ((size_t)std::min(max_len, C) + 1 + PT - 1) / PT * PT;
    const size_t nt = ra / PT, tiles = nt * (nt + 1) / 2;
    const size_t nk = prio_ldp(nprog) / PK;
    size_t sp = std::max<size_t>(64, 512 / tiles);
    sp = (sp + 7) / 8 * 8;
    sp = std::min(sp, std::max<size_t>(8, (nk + 7) / 8 * 8));
    *rows_act = ra;
    *ntiles = tiles;
    *splits = sp;
    *kchunk = (nk + sp - 1) / sp * PK;
}

extern "C" size_t syzcov_dev_prio_pos_ws_size(size_t nprog, int C, int max_len) {
    size_t ra, tiles, sp, kc;
    pos_plan(nprog, C, max_len, &ra, &tiles, &sp, &kc);
    return align_up(sp * tiles * PT * PT * 4, 256);
}

extern "C" int syzcov_dev_prio_counts_pos(const int32_t *lens, size_t nprog, int C, int max_len,
                                          int32_t *counts, void *ws, size_t ws_size,
                                          void *stream) {
    if (C <= 0 || !counts || (nprog && !lens) || max_len < 0 || max_len > C) return SYZCOV_EINVAL;
    if (nprog == 0) return 0;
    if (!ws || ws_size < syzcov_dev_prio_pos_ws_size(nprog, C, max_len)) return SYZCOV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    size_t ra, tiles, sp, kc;
    pos_plan(nprog, C, max_len, &ra, &tiles, &sp, &kc);
    const size_t ldp = prio_ldp(nprog), ldc = prio_rows(C);
    int32_t *part = (int32_t *)ws;
    const int nt = (int)(ra / PT), ones = std::min(max_len, C);
    hipLaunchKernelGGL(prio_gemm_kernel<true>, dim3((unsigned)(tiles * sp)), dim3(256), 0, s,
                       (const int8_t *)nullptr, ldp, kc, nt, (int)tiles, (int)(sp / 8), counts, ra,
                       ldc, part, lens, nprog, ones);
    hipLaunchKernelGGL(prio_reduce_kernel<PT>,
                       dim3((unsigned)((tiles * PT * PT + 255) / 256), (unsigned)std::min<size_t>(sp, 16)),
                       dim3(256), 0, s, (const int32_t *)part, sp, (int)tiles, nt, counts, ldc, ones,
                       C);
    SYZ_LAUNCH_CHECK();
    return 0;
}
