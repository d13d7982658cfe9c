// synth.hip -- top-down synthetic Multi-BRWT generated straight into the
// device image (DESIGN.md "Synthetic matrices").
//
// Law: a BRWT of the basic arity-k partitioner shape (BRWT_builders.cpp:20-31,
// pass-through of singleton groups :74-76) built from i.i.d. Bernoulli(d)
// columns (experiments/data_generation.cpp:20-29).  Given that row r reaches
// node u (u's index bit set), the children's "subtree nonzero" indicators are
// independent Bernoulli(q_c), q_c = 1 - (1-d)^cols(c), conditioned on not all
// being zero -- the conditional law of OR-ed i.i.d. columns.  The root bit is
// Bernoulli(q_root).  Each position draws ONE 64-bit hash of (seed, node,
// position) and maps it through the node's inverse-CDF table over nonzero
// child masks, so the structure is a pure function of the seed; the CPU
// oracle implements the same spec independently (oracle/brwt_oracle.cpp).
//
// The 3.7 B x 2,652 Kingsford shape (~77 G mask draws, ~127 GB image) is
// generated level by level in a few seconds; the reference's column-major
// mt19937 path would need ~1.2 TB of raw bits.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

#include "mbrwt_internal.hpp"

namespace mbrwt {

namespace {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t node_key(uint64_t seed, uint64_t key) {
    return mix64(seed ^ ((key + 1) * 0x9E3779B97F4A7C15ull));
}
constexpr uint64_t kDrawMul = 0xD1B54A32D192ED03ull;
__host__ __device__ __forceinline__ uint64_t draw(uint64_t k, uint64_t pos) {
    return mix64(k + pos * kDrawMul);
}
constexpr uint64_t kRootKey = 0xFFFFFFFFull;
constexpr uint32_t kSynthMaxArity = 12;

uint64_t prob_to_threshold(double p) {
    if (!(p > 0.0)) return 0;
    if (p >= 1.0) return UINT64_MAX;
    return (uint64_t)(p * 18446744073709551616.0);
}

// inverse-CDF thresholds over nonzero masks 1..2^a-1 (same order of
// floating-point operations as the spec; built with -ffp-contract=off)
std::vector<uint64_t> mask_table(const std::vector<double> &q) {
    const size_t a = q.size();
    const size_t nm = (1ull << a) - 1;
    std::vector<uint64_t> T(nm, UINT64_MAX);
    double prod0 = 1.0;
    for (size_t c = 0; c < a; ++c) prod0 = prod0 * (1.0 - q[c]);
    const double Z = 1.0 - prod0;
    if (!(Z > 0.0)) return T;
    double cum = 0.0;
    for (size_t k = 1; k <= nm; ++k) {
        double p = 1.0;
        for (size_t c = 0; c < a; ++c) p = p * (((k >> c) & 1) ? q[c] : (1.0 - q[c]));
        cum = cum + p / Z;
        T[k - 1] = (k == nm) ? UINT64_MAX : prob_to_threshold(cum);
    }
    return T;
}

__device__ __forceinline__ bool bern(uint64_t x, uint64_t t) { return x < t || t == UINT64_MAX; }

__device__ __forceinline__ uint32_t draw_mask(const uint64_t *__restrict__ T, uint32_t nT, uint64_t x) {
    uint32_t lo = 0, hi = nT - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (x < T[mid]) hi = mid;
        else lo = mid + 1;
    }
    return lo + 1;
}

// ---- image kernels -----------------------------------------------------

// super-root as KIND_PLANE with one child (the internal root): bits of the
// root index column, Bernoulli(q_root) per row
__global__ __launch_bounds__(256) void k_gen_root_plane(uint8_t *img, uint64_t L, uint64_t K, uint64_t T,
                                                         uint32_t stride) {
    const uint64_t nb = (L + 31) / 32;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        uint32_t bits = 0;
        for (uint32_t t = 0; t < 32; ++t) {
            const uint64_t j = b * 32 + t;
            if (j < L && bern(draw(K, j), T)) bits |= 1u << t;
        }
        *reinterpret_cast<uint2 *>(img + b * stride) = make_uint2(0u, bits);
    }
}

// super-root as KIND_MASK8 when the root is a leaf (one column)
__global__ __launch_bounds__(256) void k_gen_root_mask(uint8_t *img, uint64_t L, uint64_t K, uint64_t T,
                                                        unsigned long long *ones) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    uint64_t local = 0;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < L; j += gs) {
        const uint8_t b = bern(draw(K, j), T) ? 1 : 0;
        img[j] = b;
        local += b;
    }
    if (local) atomicAdd(ones, (unsigned long long)local);
}

// internal node with at least one internal child: KIND_PLANE blocks
template <int A>
__global__ __launch_bounds__(256) void k_gen_plane(uint8_t *img, uint64_t L, uint64_t K,
                                                   const uint64_t *__restrict__ Tg, uint32_t nT, uint32_t stride) {
    __shared__ uint64_t T[(1 << A) - 1];
    for (uint32_t i = threadIdx.x; i < nT; i += blockDim.x) T[i] = Tg[i];
    __syncthreads();
    const uint64_t nb = (L + 31) / 32;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        uint32_t bits[A];
#pragma unroll
        for (int c = 0; c < A; ++c) bits[c] = 0;
        for (uint32_t t = 0; t < 32; ++t) {
            const uint64_t j = b * 32 + t;
            if (j >= L) break;
            const uint32_t m = draw_mask(T, nT, draw(K, j));
#pragma unroll
            for (int c = 0; c < A; ++c) bits[c] |= ((m >> c) & 1u) << t;
        }
        uint8_t *blk = img + b * stride;
#pragma unroll
        for (int c = 0; c < A; ++c) *reinterpret_cast<uint2 *>(blk + 8 * c) = make_uint2(0u, bits[c]);
    }
}

// internal node whose children are all leaves: one mask per position
template <typename W, int A>
__global__ __launch_bounds__(256) void k_gen_mask(W *img, uint64_t L, uint64_t K, const uint64_t *__restrict__ Tg,
                                                  uint32_t nT, unsigned long long *ones) {
    __shared__ uint64_t T[(1 << A) - 1];
    for (uint32_t i = threadIdx.x; i < nT; i += blockDim.x) T[i] = Tg[i];
    __syncthreads();
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    uint64_t local = 0;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < L; j += gs) {
        const uint32_t m = draw_mask(T, nT, draw(K, j));
        img[j] = (W)m;
        local += (uint64_t)__builtin_popcount(m);
    }
    // wave-level reduction before the atomic
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(ones, (unsigned long long)local);
}

// root folding: the super-root image holds the root's children over ROW
// positions.  The root's own column (a temporary plane, ranks scanned) gives
// the root position j of every set row; the mask drawn at (root, j) is the
// same draw as in the unfolded image, so the structure is identical.
template <int A>
__global__ __launch_bounds__(256) void k_gen_fold_plane(uint8_t *img, uint64_t n, const uint8_t *root_img,
                                                        uint64_t K, const uint64_t *__restrict__ Tg, uint32_t nT,
                                                        uint32_t stride) {
    __shared__ uint64_t T[(1 << A) - 1];
    for (uint32_t i = threadIdx.x; i < nT; i += blockDim.x) T[i] = Tg[i];
    __syncthreads();
    const uint64_t nb = (n + 31) / 32;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        const uint2 rb = *reinterpret_cast<const uint2 *>(root_img + b * 16);
        uint32_t bits[A];
#pragma unroll
        for (int c = 0; c < A; ++c) bits[c] = 0;
        uint32_t x = rb.y;
        while (x) {
            const uint32_t t = __builtin_ctz(x);
            x &= x - 1;
            const uint64_t j = rb.x + __builtin_popcount(rb.y & ((1u << t) - 1u));
            const uint32_t m = draw_mask(T, nT, draw(K, j));
#pragma unroll
            for (int c = 0; c < A; ++c) bits[c] |= ((m >> c) & 1u) << t;
        }
        uint8_t *blk = img + b * stride;
#pragma unroll
        for (int c = 0; c < A; ++c) *reinterpret_cast<uint2 *>(blk + 8 * c) = make_uint2(0u, bits[c]);
    }
}

template <typename W, int A>
__global__ __launch_bounds__(256) void k_gen_fold_mask(W *img, uint64_t n, const uint8_t *root_img, uint64_t K,
                                                       const uint64_t *__restrict__ Tg, uint32_t nT,
                                                       unsigned long long *ones) {
    __shared__ uint64_t T[(1 << A) - 1];
    for (uint32_t i = threadIdx.x; i < nT; i += blockDim.x) T[i] = Tg[i];
    __syncthreads();
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    uint64_t local = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gs) {
        const uint2 rb = *reinterpret_cast<const uint2 *>(root_img + (r >> 5) * 16);
        const uint32_t t = r & 31;
        uint32_t m = 0;
        if ((rb.y >> t) & 1u) {
            const uint64_t j = rb.x + __builtin_popcount(rb.y & ((1u << t) - 1u));
            m = draw_mask(T, nT, draw(K, j));
        }
        img[r] = (W)m;
        local += (uint64_t)__builtin_popcount(m);
    }
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(ones, (unsigned long long)local);
}

// KIND_PACK image (mbrwt_internal.hpp) of a node whose children are MASK8
// nodes, from its temporary KIND_PLANE image (children bits + ranks): the
// mask of child c at child position jc is the same draw (child key, jc) as
// the child's own MASK8 image would hold.  Pass 0 counts the blocks that
// spill; pass 1 writes (spill lists in 128-byte slots taken atomically).
struct PackArgs {
    const uint64_t *T[8];
    uint32_t nT[8];
    uint64_t K[8];
};

template <int A>
__global__ __launch_bounds__(256) void k_gen_pack(uint8_t *img, uint64_t L, const uint8_t *plane, uint32_t pstride,
                                                  PackArgs args, uint8_t *spill, unsigned long long *spill_ctr,
                                                  unsigned long long *ones, int pass) {
    __shared__ uint64_t T[A][255];
    for (int c = 0; c < A; ++c)
        for (uint32_t i = threadIdx.x; i < args.nT[c]; i += blockDim.x) T[c][i] = args.T[c][i];
    __syncthreads();
    const uint64_t nb = (L + kPackSpan - 1) / kPackSpan;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    uint64_t local = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        const uint8_t *pb = plane + (b >> 1) * pstride;
        const uint32_t half = (uint32_t)(b & 1) * 16;
        uint32_t total = 0;
        uint32_t bits[A];
#pragma unroll
        for (int c = 0; c < A; ++c) {
            bits[c] = (reinterpret_cast<const uint2 *>(pb + 8 * c)->y >> half) & 0xFFFFu;
            total += __builtin_popcount(bits[c]);
        }
        if (pass == 0) {
            if (total > kPackArea) atomicAdd(spill_ctr, 1ull);
            continue;
        }
        uint8_t *blk = img + b * kPackBlock;
        uint8_t *out = nullptr;
        if (total > kPackArea) {
            out = spill + atomicAdd(spill_ctr, 1ull) * 128;
            const uint64_t addr = (uint64_t)(uintptr_t)out;
            for (uint32_t k = 0; k < 8; ++k) blk[pack_area_byte(k)] = (uint8_t)(addr >> (8 * k));
        }
        uint32_t o = 0;
#pragma unroll
        for (int c = 0; c < A; ++c) {
            const uint2 rb = *reinterpret_cast<const uint2 *>(pb + 8 * c);
            *reinterpret_cast<uint16_t *>(blk + 16 * (c / 2) + 2 * (c % 2)) = (uint16_t)bits[c];
            for (uint32_t x = bits[c]; x; x &= x - 1) {
                const uint32_t t = half + __builtin_ctz(x);
                const uint64_t jc = rb.x + __builtin_popcount(rb.y & ((1u << t) - 1u));
                const uint32_t m = draw_mask(T[c], args.nT[c], draw(args.K[c], jc));
                local += __builtin_popcount(m);
                if (out) out[o] = (uint8_t)m;
                else blk[pack_area_byte(o)] = (uint8_t)m;
                ++o;
            }
        }
    }
    if (pass == 1) {
        for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off);
        if ((threadIdx.x & 63) == 0 && local) atomicAdd(ones, (unsigned long long)local);
    }
}

template <int A>
void launch_pack(uint8_t *img, uint64_t L, const uint8_t *plane, uint32_t pstride, const PackArgs &args,
                 uint8_t *spill, unsigned long long *ctr, unsigned long long *ones, int pass, hipStream_t s) {
    const uint64_t nb = (L + kPackSpan - 1) / kPackSpan;
    hipLaunchKernelGGL(k_gen_pack<A>, dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nb + 255) / 256, 65536))),
                       dim3(256), 0, s, img, L, plane, pstride, args, spill, ctr, ones, pass);
}
using PackFn = void (*)(uint8_t *, uint64_t, const uint8_t *, uint32_t, const PackArgs &, uint8_t *,
                        unsigned long long *, unsigned long long *, int, hipStream_t);
PackFn pack_fn(uint32_t a) {
    static const PackFn t[] = {nullptr, launch_pack<1>, launch_pack<2>, launch_pack<3>, launch_pack<4>,
                               launch_pack<5>, launch_pack<6>, launch_pack<7>, launch_pack<8>};
    return a >= 1 && a <= 8 ? t[a] : nullptr;
}

// KIND_PACK2 image (mbrwt_internal.hpp) of node u from temporary KIND_PLANE
// images of u (its children A's bits + ranks over u's positions) and of
// every A (A's MASK8 children B's bits + ranks over A's positions); the leaf
// mask of B at B's position jB is the same draw (B's key, jB) as B's own
// MASK8 image would hold.  One thread per block of S positions (the node's
// span).  Pass 0 sums the bytes of the spill lists; pass 1 writes (lists
// placed atomically).
struct Pack2Args {
    const uint8_t *uplane;
    uint32_t ustride;
    uint32_t a;                  // u's arity
    const uint8_t *aplane[8];    // A's temporary planes
    uint32_t astride[8];
    uint32_t aarity[8];
    uint64_t KB[64];             // key of B = child b of A: [8 * A + b]
    uint8_t tB[64];              // table slot of B
    const uint64_t *T[4];        // distinct tables of the B nodes (<= 4)
    uint32_t nT[4];
};

__device__ __forceinline__ uint32_t plane_bit_rank(const uint8_t *plane, uint32_t stride, uint32_t c, uint64_t j,
                                                   uint32_t &rank) {
    const uint2 e = *reinterpret_cast<const uint2 *>(plane + (j >> 5) * stride + 8 * c);
    const uint32_t t = (uint32_t)(j & 31);
    rank = e.x + (uint32_t)__builtin_popcount(e.y & ((1u << t) - 1u));
    return (e.y >> t) & 1u;
}

__global__ __launch_bounds__(256) void k_gen_pack2(uint8_t *img, uint64_t L, uint32_t S, Pack2Args args,
                                                   uint8_t *spill, unsigned long long *spill_ctr,
                                                   unsigned long long *ones, int pass) {
    __shared__ uint64_t T[4][255];
    for (int k = 0; k < 4; ++k)
        for (uint32_t i = threadIdx.x; i < args.nT[k]; i += blockDim.x) T[k][i] = args.T[k][i];
    __syncthreads();
    const uint64_t nb = (L + S - 1) / S;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    uint64_t local = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        // record bytes of the block
        uint32_t size = 0;
        for (uint32_t t = 0; t < S; ++t) {
            const uint64_t j = b * S + t;
            if (j >= L) break;
            size += 1;
            for (uint32_t A = 0; A < args.a; ++A) {
                uint32_t jA;
                if (!plane_bit_rank(args.uplane, args.ustride, A, j, jA)) continue;
                size += 1;
                for (uint32_t B = 0; B < args.aarity[A]; ++B) {
                    uint32_t jB;
                    size += plane_bit_rank(args.aplane[A], args.astride[A], B, jA, jB);
                }
            }
        }
        const bool spills = size > pack2_inline(S);
        const uint32_t list_bytes = (2 * (S + 1) + size + 15) & ~15u;
        if (pass == 0) {
            if (spills) atomicAdd(spill_ctr, (unsigned long long)list_bytes);
            if (spills && size > kPack2Block) {  // some record may exceed 64 bytes: check each
                for (uint32_t t = 0; t < S; ++t) {
                    const uint64_t j = b * S + t;
                    if (j >= L) break;
                    uint32_t rs = 1;
                    for (uint32_t A = 0; A < args.a; ++A) {
                        uint32_t jA;
                        if (!plane_bit_rank(args.uplane, args.ustride, A, j, jA)) continue;
                        rs += 1;
                        for (uint32_t B = 0; B < args.aarity[A]; ++B) {
                            uint32_t jB;
                            rs += plane_bit_rank(args.aplane[A], args.astride[A], B, jA, jB);
                        }
                    }
                    if (rs > kPack2Block) atomicAdd(spill_ctr + 1, 1ull);
                }
            }
            continue;
        }
        uint8_t *blk = img + b * kPack2Block;
        uint8_t *dst;
        uint32_t hdr;  // start[t] = hdr + offset in the record bytes
        if (spills) {
            uint8_t *list = spill + atomicAdd(spill_ctr, (unsigned long long)list_bytes);
            const uint64_t addr = (uint64_t)(uintptr_t)list;
            for (uint32_t k = 0; k < 8; ++k) {
                blk[k] = 0;
                blk[8 + k] = (uint8_t)(addr >> (8 * k));
            }
            dst = list + 2 * (S + 1);  // u16 start[S+1], then the records
            hdr = 2 * (S + 1);
        } else {
            dst = blk + S;
            hdr = S;
        }
        uint32_t o = 0;
        for (uint32_t t = 0; t < S; ++t) {
            const uint64_t j = b * S + t;
            if (spills) *reinterpret_cast<uint16_t *>(dst - 2 * (S + 1) + 2 * t) = (uint16_t)(hdr + o);
            else blk[t] = (uint8_t)(hdr + o);
            if (j >= L) continue;
            uint32_t m2 = 0, jA[8], m1[8];
            for (uint32_t A = 0; A < args.a; ++A) m2 |= plane_bit_rank(args.uplane, args.ustride, A, j, jA[A]) << A;
            dst[o++] = (uint8_t)m2;
            for (uint32_t A = 0; A < args.a; ++A) {
                m1[A] = 0;
                if (!((m2 >> A) & 1u)) continue;
                uint32_t r;
                for (uint32_t B = 0; B < args.aarity[A]; ++B)
                    m1[A] |= plane_bit_rank(args.aplane[A], args.astride[A], B, jA[A], r) << B;
                dst[o++] = (uint8_t)m1[A];
            }
            for (uint32_t A = 0; A < args.a; ++A) {
                for (uint32_t x = m1[A]; x; x &= x - 1) {
                    const uint32_t B = (uint32_t)__builtin_ctz(x);
                    uint32_t jB;
                    (void)plane_bit_rank(args.aplane[A], args.astride[A], B, jA[A], jB);
                    const uint32_t ti = args.tB[8 * A + B];
                    const uint32_t lm = draw_mask(T[ti], args.nT[ti], draw(args.KB[8 * A + B], jB));
                    local += (uint64_t)__builtin_popcount(lm);
                    dst[o++] = (uint8_t)lm;
                }
            }
        }
        if (spills) *reinterpret_cast<uint16_t *>(dst - 2 * (S + 1) + 2 * S) = (uint16_t)(hdr + o);  // end
    }
    if (pass == 1) {
        for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off);
        if ((threadIdx.x & 63) == 0 && local) atomicAdd(ones, (unsigned long long)local);
    }
}

// KIND_PACKT image (mbrwt_internal.hpp) of a root child u from temporary
// KIND_PLANE images of the internal nodes of u's subtree that have internal
// children; the masks of all-leaf nodes are drawn at their positions (the
// same draw (key, position) as their own MASK images would hold).  One
// thread per block of S positions walks each position's DFS record; pass 0
// sums the spill-list bytes and counts records over 64 bytes, pass 1 writes.
struct GenNode {
    uint64_t K;
    const uint64_t *T;
    const uint8_t *plane;  // temporary KIND_PLANE image, null = all children leaves (masks drawn)
    uint32_t nT, stride, arity, child0;  // child0: index of child 0 in the child table
};
constexpr uint32_t kGenLeaf = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t gen_mask(const GenNode &v, uint64_t jv) {
    if (!v.plane) return draw_mask(v.T, v.nT, draw(v.K, jv));
    uint32_t m = 0, r;
    for (uint32_t c = 0; c < v.arity; ++c) m |= plane_bit_rank(v.plane, v.stride, c, jv, r) << c;
    return m;
}

// the DFS record of u (gen node 0) at position j: put(mask, arity) per
// visited internal node in pre-order; false past kPacktMaxDepth levels
template <typename Put>
__device__ bool gen_packt_record(const GenNode *__restrict__ gn, const uint32_t *__restrict__ gch, uint64_t j, Put put,
                                 uint64_t &leaves) {
    uint32_t nd[kPacktMaxDepth], rem[kPacktMaxDepth];
    uint64_t ps[kPacktMaxDepth];
    const GenNode u = gn[0];
    const uint32_t m = gen_mask(u, j);
    put(m, u.arity);
    nd[0] = 0;
    ps[0] = j;
    rem[0] = m;
    int sp = 1;
    while (sp) {
        const int t = sp - 1;
        if (!rem[t]) {
            --sp;
            continue;
        }
        const uint32_t c = (uint32_t)__builtin_ctz(rem[t]);
        rem[t] &= rem[t] - 1;
        const GenNode &v = gn[nd[t]];
        const uint32_t ch = gch[v.child0 + c];
        if (ch == kGenLeaf) {
            ++leaves;
            continue;
        }
        uint32_t jc;
        (void)plane_bit_rank(v.plane, v.stride, c, ps[t], jc);
        const GenNode w = gn[ch];
        const uint32_t mw = gen_mask(w, jc);
        put(mw, w.arity);
        if (sp == (int)kPacktMaxDepth) return false;
        nd[sp] = ch;
        ps[sp] = jc;
        rem[sp] = mw;
        ++sp;
    }
    return true;
}

__global__ __launch_bounds__(256) void k_gen_packt(uint8_t *img, uint64_t L, uint32_t S, const GenNode *gn,
                                                   const uint32_t *gch, uint8_t *spill,
                                                   unsigned long long *spill_ctr, unsigned long long *ones, int pass) {
    const uint64_t nb = (L + S - 1) / S;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    uint64_t local = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gs) {
        uint32_t size = 0;
        bool big = false;
        for (uint32_t t = 0; t < S; ++t) {
            const uint64_t j = b * S + t;
            if (j >= L) break;
            uint32_t rs = 1;  // the label count
            uint64_t labels = 0;
            if (!gen_packt_record(gn, gch, j, [&](uint32_t, uint32_t a) { rs += packt_mask_bytes(a); }, labels))
                big = true;
            size += rs;
            big |= rs > kPack2Block || labels > 255;
        }
        const bool spills = size > pack2_inline(S);
        const uint32_t list_bytes = (2 * (S + 1) + size + 15) & ~15u;
        if (pass == 0) {
            if (spills) atomicAdd(spill_ctr, (unsigned long long)list_bytes);
            if (big) atomicAdd(spill_ctr + 1, 1ull);
            continue;
        }
        uint8_t *blk = img + b * kPack2Block;
        uint8_t *dst;
        uint32_t hdr;
        if (spills) {
            uint8_t *list = spill + atomicAdd(spill_ctr, (unsigned long long)list_bytes);
            const uint64_t addr = (uint64_t)(uintptr_t)list;
            for (uint32_t k = 0; k < 8; ++k) {
                blk[k] = 0;
                blk[8 + k] = (uint8_t)(addr >> (8 * k));
            }
            dst = list + 2 * (S + 1);
            hdr = 2 * (S + 1);
        } else {
            dst = blk + S;
            hdr = S;
        }
        uint32_t o = 0;
        for (uint32_t t = 0; t < S; ++t) {
            const uint64_t j = b * S + t;
            if (spills) *reinterpret_cast<uint16_t *>(dst - 2 * (S + 1) + 2 * t) = (uint16_t)(hdr + o);
            else blk[t] = (uint8_t)(hdr + o);
            if (j >= L) continue;
            const uint32_t at = o++;
            uint64_t labels = 0;
            (void)gen_packt_record(
                gn, gch, j,
                [&](uint32_t m, uint32_t a) {
                    dst[o++] = (uint8_t)m;
                    if (a > 8) dst[o++] = (uint8_t)(m >> 8);
                },
                labels);
            dst[at] = (uint8_t)labels;
            local += labels;
        }
        if (spills) *reinterpret_cast<uint16_t *>(dst - 2 * (S + 1) + 2 * S) = (uint16_t)(hdr + o);  // end
    }
    if (pass == 1) {
        for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off);
        if ((threadIdx.x & 63) == 0 && local) atomicAdd(ones, (unsigned long long)local);
    }
}

// ---- per-child rank scan over the blocks of a KIND_PLANE image ----------
constexpr int kScanTile = 256;  // blocks per tile (one thread per block)

__global__ __launch_bounds__(kScanTile) void k_tile_sums(const uint8_t *img, uint64_t nb, uint32_t a,
                                                         uint32_t stride, uint64_t *tile_sums) {
    typedef hipcub::BlockReduce<uint32_t, kScanTile> BR;
    __shared__ typename BR::TempStorage tmp;
    const uint64_t tile = blockIdx.x;
    const uint64_t b = tile * kScanTile + threadIdx.x;
    for (uint32_t c = 0; c < a; ++c) {
        uint32_t v = 0;
        if (b < nb) v = __builtin_popcount(reinterpret_cast<const uint2 *>(img + b * stride + 8 * c)->y);
        const uint32_t s = BR(tmp).Sum(v);
        if (threadIdx.x == 0) tile_sums[tile * a + c] = s;
        __syncthreads();
    }
}

// exclusive scan of tile sums per child (one workgroup per child), totals out
__global__ __launch_bounds__(1024) void k_scan_tiles(uint64_t *tile_sums, uint64_t ntiles, uint32_t a,
                                                     uint64_t *totals) {
    typedef hipcub::BlockScan<uint64_t, 1024> BS;
    __shared__ typename BS::TempStorage tmp;
    __shared__ uint64_t carry;
    const uint32_t c = blockIdx.x;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint64_t base = 0; base < ntiles; base += 1024) {
        const uint64_t t = base + threadIdx.x;
        const uint64_t v = t < ntiles ? tile_sums[t * a + c] : 0;
        uint64_t ex, agg;
        BS(tmp).ExclusiveSum(v, ex, agg);
        const uint64_t cr = carry;
        if (t < ntiles) tile_sums[t * a + c] = cr + ex;
        __syncthreads();
        if (threadIdx.x == 0) carry = cr + agg;
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[c] = carry;
}

__global__ __launch_bounds__(kScanTile) void k_write_ranks(uint8_t *img, uint64_t nb, uint32_t a, uint32_t stride,
                                                           const uint64_t *tile_offsets) {
    typedef hipcub::BlockScan<uint32_t, kScanTile> BS;
    __shared__ typename BS::TempStorage tmp;
    const uint64_t tile = blockIdx.x;
    const uint64_t b = tile * kScanTile + threadIdx.x;
    for (uint32_t c = 0; c < a; ++c) {
        uint2 *e = reinterpret_cast<uint2 *>(img + b * stride + 8 * c);
        uint32_t v = 0;
        if (b < nb) v = __builtin_popcount(e->y);
        uint32_t ex;
        BS(tmp).ExclusiveSum(v, ex);
        if (b < nb) e->x = (uint32_t)(tile_offsets[tile * a + c] + ex);
        __syncthreads();
    }
}

int launch_grid(uint64_t items) { return (int)std::max<uint64_t>(1, std::min<uint64_t>((items + 255) / 256, 65536)); }

// rank scan of a KIND_PLANE image; returns per-child totals (lengths of the
// children's index columns)
int plane_scan(uint8_t *img, uint64_t L, uint32_t a, uint32_t stride, std::vector<uint64_t> &totals,
               hipStream_t s) {
    const uint64_t nb = (L + 31) / 32;
    const uint64_t ntiles = std::max<uint64_t>(1, (nb + kScanTile - 1) / kScanTile);
    uint64_t *d_tiles = nullptr, *d_tot = nullptr;
    MBRWT_HIP(hipMalloc(&d_tiles, ntiles * a * sizeof(uint64_t)));
    MBRWT_HIP(hipMalloc(&d_tot, a * sizeof(uint64_t)));
    if (nb) {
        hipLaunchKernelGGL(k_tile_sums, dim3((unsigned)ntiles), dim3(kScanTile), 0, s, img, nb, a, stride, d_tiles);
        MBRWT_HIP(hipGetLastError());
    } else {
        MBRWT_HIP(hipMemsetAsync(d_tiles, 0, ntiles * a * sizeof(uint64_t), s));
    }
    hipLaunchKernelGGL(k_scan_tiles, dim3(a), dim3(1024), 0, s, d_tiles, ntiles, a, d_tot);
    MBRWT_HIP(hipGetLastError());
    if (nb) {
        hipLaunchKernelGGL(k_write_ranks, dim3((unsigned)ntiles), dim3(kScanTile), 0, s, img, nb, a, stride, d_tiles);
        MBRWT_HIP(hipGetLastError());
    }
    totals.assign(a, 0);
    MBRWT_HIP(hipMemcpyAsync(totals.data(), d_tot, a * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    MBRWT_HIP(hipFree(d_tiles));
    MBRWT_HIP(hipFree(d_tot));
    return MBRWT_OK;
}

struct ShapeNode {
    std::vector<uint32_t> children;
    uint64_t cols = 0;
    uint32_t column = UINT32_MAX;  // leaves
};

// basic-partitioner shape in BFS numbering (node 0 = root)
std::vector<ShapeNode> basic_shape(uint64_t m, uint32_t arity) {
    std::vector<ShapeNode> all;
    std::vector<uint32_t> cur;
    for (uint64_t i = 0; i < m; ++i) {
        ShapeNode s;
        s.cols = 1;
        s.column = (uint32_t)i;
        all.push_back(s);
        cur.push_back((uint32_t)i);
    }
    while (cur.size() > 1) {
        std::vector<uint32_t> next;
        for (size_t b = 0; b < cur.size(); b += arity) {
            const size_t e = std::min<size_t>(cur.size(), b + arity);
            if (e - b == 1) {
                next.push_back(cur[b]);
                continue;
            }
            ShapeNode p;
            for (size_t i = b; i < e; ++i) {
                p.children.push_back(cur[i]);
                p.cols += all[cur[i]].cols;
            }
            all.push_back(p);
            next.push_back((uint32_t)all.size() - 1);
        }
        cur.swap(next);
    }
    std::vector<uint32_t> order{cur[0]};
    for (size_t h = 0; h < order.size(); ++h)
        for (uint32_t c : all[order[h]].children) order.push_back(c);
    std::vector<uint32_t> newid(all.size());
    for (size_t i = 0; i < order.size(); ++i) newid[order[i]] = (uint32_t)i;
    std::vector<ShapeNode> bfs;
    bfs.reserve(order.size());
    for (uint32_t o : order) {
        ShapeNode s = all[o];
        for (auto &c : s.children) c = newid[c];
        bfs.push_back(s);
    }
    return bfs;
}

template <int A>
void launch_plane(uint8_t *img, uint64_t L, uint64_t K, const uint64_t *T, uint32_t nT, uint32_t stride,
                  hipStream_t s) {
    hipLaunchKernelGGL(k_gen_plane<A>, dim3(launch_grid((L + 31) / 32)), dim3(256), 0, s, img, L, K, T, nT, stride);
}
template <typename W, int A>
void launch_mask(uint8_t *img, uint64_t L, uint64_t K, const uint64_t *T, uint32_t nT, unsigned long long *ones,
                 hipStream_t s) {
    hipLaunchKernelGGL((k_gen_mask<W, A>), dim3(launch_grid(L)), dim3(256), 0, s, reinterpret_cast<W *>(img), L, K,
                       T, nT, ones);
}

template <int A>
void launch_fold_plane(uint8_t *img, uint64_t n, const uint8_t *root, uint64_t K, const uint64_t *T, uint32_t nT,
                       uint32_t stride, unsigned long long *, hipStream_t s) {
    hipLaunchKernelGGL(k_gen_fold_plane<A>, dim3(launch_grid((n + 31) / 32)), dim3(256), 0, s, img, n, root, K, T,
                       nT, stride);
}
template <typename W, int A>
void launch_fold_mask(uint8_t *img, uint64_t n, const uint8_t *root, uint64_t K, const uint64_t *T, uint32_t nT,
                      uint32_t, unsigned long long *ones, hipStream_t s) {
    hipLaunchKernelGGL((k_gen_fold_mask<W, A>), dim3(launch_grid(n)), dim3(256), 0, s, reinterpret_cast<W *>(img), n,
                       root, K, T, nT, ones);
}
using FoldFn = void (*)(uint8_t *, uint64_t, const uint8_t *, uint64_t, const uint64_t *, uint32_t, uint32_t,
                        unsigned long long *, hipStream_t);
FoldFn fold_fn(uint32_t a, bool plane) {
    static const FoldFn tp[] = {nullptr, launch_fold_plane<1>, launch_fold_plane<2>, launch_fold_plane<3>,
                                launch_fold_plane<4>, launch_fold_plane<5>, launch_fold_plane<6>,
                                launch_fold_plane<7>, launch_fold_plane<8>, launch_fold_plane<9>,
                                launch_fold_plane<10>, launch_fold_plane<11>, launch_fold_plane<12>};
    static const FoldFn tm[] = {nullptr,
                                launch_fold_mask<uint8_t, 1>,   launch_fold_mask<uint8_t, 2>,
                                launch_fold_mask<uint8_t, 3>,   launch_fold_mask<uint8_t, 4>,
                                launch_fold_mask<uint8_t, 5>,   launch_fold_mask<uint8_t, 6>,
                                launch_fold_mask<uint8_t, 7>,   launch_fold_mask<uint8_t, 8>,
                                launch_fold_mask<uint16_t, 9>,  launch_fold_mask<uint16_t, 10>,
                                launch_fold_mask<uint16_t, 11>, launch_fold_mask<uint16_t, 12>};
    if (a > kSynthMaxArity) return nullptr;
    return plane ? tp[a] : tm[a];
}

using PlaneFn = void (*)(uint8_t *, uint64_t, uint64_t, const uint64_t *, uint32_t, uint32_t, hipStream_t);
using MaskFn = void (*)(uint8_t *, uint64_t, uint64_t, const uint64_t *, uint32_t, unsigned long long *, hipStream_t);

PlaneFn plane_fn(uint32_t a) {
    static const PlaneFn t[] = {nullptr, launch_plane<1>, launch_plane<2>, launch_plane<3>, launch_plane<4>,
                                launch_plane<5>, launch_plane<6>, launch_plane<7>, launch_plane<8>, launch_plane<9>,
                                launch_plane<10>, launch_plane<11>, launch_plane<12>};
    return a <= kSynthMaxArity ? t[a] : nullptr;
}
MaskFn mask_fn(uint32_t a) {
    static const MaskFn t[] = {nullptr,
                               launch_mask<uint8_t, 1>,  launch_mask<uint8_t, 2>,   launch_mask<uint8_t, 3>,
                               launch_mask<uint8_t, 4>,  launch_mask<uint8_t, 5>,   launch_mask<uint8_t, 6>,
                               launch_mask<uint8_t, 7>,  launch_mask<uint8_t, 8>,   launch_mask<uint16_t, 9>,
                               launch_mask<uint16_t, 10>, launch_mask<uint16_t, 11>, launch_mask<uint16_t, 12>};
    return a <= kSynthMaxArity ? t[a] : nullptr;
}

// a given tree shape (mbrwt_shape_desc) -> ShapeNode list; empty + error on a malformed one
std::vector<ShapeNode> shape_from_desc(const mbrwt_shape_desc &sd, uint64_t m) {
    const uint32_t N = sd.num_nodes;
    std::vector<ShapeNode> sh(N);
    if (!N || !sd.num_children || !sd.first_child || !sd.leaf_column) return {};
    std::vector<uint8_t> seen(N, 0), col_seen(m, 0);
    uint64_t leaves = 0;
    for (uint32_t u = 0; u < N; ++u) {
        const uint32_t a = sd.num_children[u];
        if (a == 0) {
            const uint32_t col = sd.leaf_column[u];
            if (col >= m || col_seen[col]++) return {};
            sh[u].column = col;
            ++leaves;
            continue;
        }
        if (a > kSynthMaxArity || sd.first_child[u] <= u || (uint64_t)sd.first_child[u] + a > N) return {};
        for (uint32_t c = 0; c < a; ++c) {
            if (seen[sd.first_child[u] + c]++) return {};
            sh[u].children.push_back(sd.first_child[u] + c);
        }
    }
    if (leaves != m) return {};
    for (uint32_t u = N; u-- > 0;) {
        if (sh[u].children.empty()) {
            sh[u].cols = 1;
            continue;
        }
        for (uint32_t c : sh[u].children) sh[u].cols += sh[c].cols;
    }
    return sh;
}

}  // namespace

// KIND_PACKT images of the folded root's internal children (mbrwt_internal.hpp),
// unless every root child has the PACK2 shape (k_traverse_p2w).  A subtree
// taller than kPacktMaxDepth, or one whose records would exceed 64 bytes,
// stays for the per-node generation.  Children lengths of the root's
// children come from the fold; the rest from the temporary planes' scans.
static int synth_packt(const std::vector<ShapeNode> &shape, const std::vector<double> &q, const std::vector<uint64_t *> &node_T,
                const std::vector<uint64_t> &keys, Tree &tree, std::vector<bool> &in_pack, unsigned long long *d_ctr,
                unsigned long long *d_ones, hipStream_t s) {
    const auto &root = shape[0].children;
    auto internal = [&](uint32_t v) { return !shape[v].children.empty(); };
    auto p2_struct = [&](uint32_t u) {
        if (!internal(u) || shape[u].children.size() > 8 || !pack2_enabled()) return false;
        for (uint32_t a : shape[u].children) {
            if (!internal(a) || shape[a].children.size() > 8) return false;
            for (uint32_t b : shape[a].children) {
                if (!internal(b) || shape[b].children.size() > 8) return false;
                for (uint32_t l : shape[b].children)
                    if (internal(l)) return false;
            }
        }
        return true;
    };
    if (std::all_of(root.begin(), root.end(), p2_struct)) return MBRWT_OK;
    int rc = MBRWT_OK;
    for (uint32_t u : root) {
        if (!internal(u) || !(q[u] > 0.0)) continue;
        // the subtree's internal nodes (BFS), their depth and arity bounds
        std::vector<uint32_t> inner{u}, lvl{1};
        bool ok = true;
        for (size_t h = 0; h < inner.size() && ok; ++h) {
            const auto &sh = shape[inner[h]];
            ok = sh.children.size() <= std::min<uint32_t>(kPacktMaxArity, kSynthMaxArity) && lvl[h] <= kPacktMaxDepth;
            for (uint32_t c : sh.children)
                if (internal(c)) {
                    inner.push_back(c);
                    lvl.push_back(lvl[h] + 1);
                }
        }
        if (!ok) continue;
        std::vector<uint32_t> loc(shape.size(), kGenLeaf);
        for (uint32_t i = 0; i < inner.size(); ++i) loc[inner[i]] = i;
        std::vector<GenNode> gn(inner.size());
        std::vector<uint32_t> gch;
        std::vector<void *> tmps;
        auto free_tmps = [&]() {
            for (void *t : tmps) (void)hipFree(t);
            tmps.clear();
        };
        double rec = 0.0;
        for (uint32_t i = 0; i < inner.size() && !rc; ++i) {
            const uint32_t v = inner[i];
            const auto &sh = shape[v];
            const uint32_t a = (uint32_t)sh.children.size();
            const DevNode &vd = tree.nodes[v + 1];
            GenNode &g = gn[i];
            g.K = keys[v];
            g.T = node_T[v];
            g.nT = (1u << a) - 1;
            g.arity = a;
            g.child0 = (uint32_t)gch.size();
            g.plane = nullptr;
            g.stride = 0;
            rec += q[v] / q[u] * packt_mask_bytes(a);
            bool all_leaves = true;
            for (uint32_t c : sh.children) {
                gch.push_back(loc[c]);
                all_leaves &= !internal(c);
            }
            if (all_leaves) continue;
            const uint32_t stride = plane_stride(a);
            const uint64_t L = vd.length, bytes = ((L + 31) / 32) * stride + kImagePad;
            void *t = nullptr;
            if (hipMalloc(&t, bytes) != hipSuccess) {
                rc = MBRWT_ERR_NOMEM;
                break;
            }
            tmps.push_back(t);
            (void)hipMemsetAsync(t, 0, bytes, s);
            uint8_t *pl = reinterpret_cast<uint8_t *>(t);
            plane_fn(a)(pl, L, g.K, g.T, g.nT, stride, s);
            std::vector<uint64_t> tot;
            if ((rc = plane_scan(pl, L, a, stride, tot, s))) break;
            for (uint32_t c = 0; c < a; ++c)
                if (internal(sh.children[c])) tree.nodes[sh.children[c] + 1].length = tot[c];
            g.plane = pl;
            g.stride = stride;
        }
        GenNode *d_gn = nullptr;
        uint32_t *d_gch = nullptr;
        if (!rc && (hipMalloc(&d_gn, gn.size() * sizeof(GenNode)) != hipSuccess ||
                    hipMalloc(&d_gch, gch.size() * 4) != hipSuccess ||
                    hipMemcpyAsync(d_gn, gn.data(), gn.size() * sizeof(GenNode), hipMemcpyHostToDevice, s) != hipSuccess ||
                    hipMemcpyAsync(d_gch, gch.data(), gch.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess))
            rc = MBRWT_ERR_NOMEM;
        auto done = [&]() {
            (void)hipStreamSynchronize(s);
            free_tmps();
            if (d_gn) (void)hipFree(d_gn);
            if (d_gch) (void)hipFree(d_gch);
        };
        if (rc) {
            done();
            return rc;
        }
        DevNode &dn = tree.nodes[u + 1];
        const uint64_t L = dn.length;
        uint32_t S = 1;  // the largest span whose expected block (header + records with counts) fits
        for (uint32_t span = kPack2MaxSpan; span >= 2; --span)
            if (span * (rec + 2.0) <= 56.0) {
                S = span;
                break;
            }
        const uint64_t nb = (L + S - 1) / S;
        (void)hipMemsetAsync(d_ctr, 0, 2 * sizeof(unsigned long long), s);
        hipLaunchKernelGGL(k_gen_packt, dim3(launch_grid(nb)), dim3(256), 0, s, nullptr, L, S, d_gn, d_gch, nullptr,
                           d_ctr, d_ones, 0);
        unsigned long long ctr[2] = {0, 0};
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(ctr, d_ctr, sizeof(ctr), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            done();
            return MBRWT_ERR_DEVICE;
        }
        if (ctr[1]) {  // a record over 64 bytes: this subtree is generated node by node
            done();
            continue;
        }
        auto alloc = [&](uint64_t bytes) -> uint8_t * {
            void *p = nullptr;
            if (hipMalloc(&p, bytes + kImagePad) != hipSuccess) return nullptr;
            (void)hipMemsetAsync(p, 0, bytes + kImagePad, s);
            tree.images.push_back(p);
            tree.image_bytes += bytes + kImagePad;
            return reinterpret_cast<uint8_t *>(p);
        };
        uint8_t *spill = ctr[0] ? alloc(ctr[0]) : nullptr;
        uint8_t *img = alloc(nb * kPack2Block);
        if (!img || (ctr[0] && !spill)) {
            done();
            return MBRWT_ERR_NOMEM;
        }
        (void)hipMemsetAsync(d_ctr, 0, sizeof(unsigned long long), s);
        hipLaunchKernelGGL(k_gen_packt, dim3(launch_grid(nb)), dim3(256), 0, s, img, L, S, d_gn, d_gch, spill, d_ctr,
                           d_ones, 1);
        if (hipGetLastError() != hipSuccess) {
            done();
            return MBRWT_ERR_DEVICE;
        }
        done();
        dn.kind = KIND_PACKT;
        dn.stride = S;
        dn.base = (uint64_t)(uintptr_t)img;
        for (uint32_t v : inner) {
            in_pack[v] = true;
            if (v == u) continue;
            DevNode &vd = tree.nodes[v + 1];
            vd.kind = KIND_PACKT_IN;
            vd.base = 0;
            vd.stride = 0;
        }
    }
    return MBRWT_OK;
}

int build_synthetic(const mbrwt_synth_desc &desc, const mbrwt_shape_desc *shape_desc, int device, Tree &tree,
                    hipStream_t s, const SynthShard *shard) {
    MBRWT_HIP(hipSetDevice(device));
    tree = Tree();
    const uint64_t n = desc.num_rows, m = desc.num_columns;
    const double d = desc.density;
    if ((!shape_desc && (desc.arity < 2 || desc.arity > kSynthMaxArity)) || !(d >= 0.0 && d <= 1.0)) {
        set_error("synthetic: arity must be in [2,12] and density in [0,1]");
        return MBRWT_ERR_INVALID;
    }
    if (n > kMaxRows) {
        set_error("synthetic: num_rows >= 2^32 is not supported by this build");
        return MBRWT_ERR_UNSUPPORTED;
    }
    tree.num_rows = n;
    tree.num_columns = m;
    if (m == 0) {
        tree.num_rows = 0;
        return finalize_tree(tree);
    }
    const auto shape = shape_desc ? shape_from_desc(*shape_desc, m) : basic_shape(m, desc.arity);
    if (shape.empty()) {
        set_error("synthetic: malformed shape (BFS order, arity <= 12, leaves = num_columns, distinct columns)");
        return MBRWT_ERR_INVALID;
    }
    const uint32_t N = (uint32_t)shape.size();
    tree.num_nodes = N;
    std::vector<double> q(N);
    for (uint32_t u = 0; u < N; ++u) q[u] = 1.0 - std::pow(1.0 - d, (double)shape[u].cols);
    // node keys; a row shard starting at row0 whose nodes start at positions
    // pos0[u] draws H(K, pos0 + j) = mix64((K + pos0 * kDrawMul) + j * kDrawMul):
    // the same bits as the unsharded tree, through a shifted key
    std::vector<uint64_t> keys(N);
    for (uint32_t u = 0; u < N; ++u)
        keys[u] = node_key(desc.seed, u) + (shard && u < shard->pos0.size() ? shard->pos0[u] : 0) * kDrawMul;
    const uint64_t root_key = node_key(desc.seed, kRootKey) + (shard ? shard->row0 : 0) * kDrawMul;

    tree.nodes.assign(N + 1, DevNode{});
    for (uint32_t u = 0; u < N; ++u) {
        DevNode &dn = tree.nodes[u + 1];
        const auto &sh = shape[u];
        if (sh.children.empty()) {
            dn.kind = KIND_LEAF;
            dn.label = sh.column;
            continue;
        }
        bool all_leaves = true;
        for (uint32_t c : sh.children) all_leaves &= shape[c].children.empty();
        dn.arity = (uint16_t)sh.children.size();
        dn.first_child = sh.children[0] + 1;
        dn.label = UINT32_MAX;
        dn.kind = all_leaves ? mask_kind(dn.arity) : KIND_PLANE;
        if (dn.kind == KIND_PLANE) dn.stride = std::max<uint32_t>(16, plane_stride(dn.arity));
        tree.max_arity = std::max<uint32_t>(tree.max_arity, dn.arity);
    }
    // per-node inverse-CDF tables, deduplicated by the children's q profile
    std::map<std::vector<double>, uint64_t *> tables;
    std::vector<uint64_t *> node_T(N, nullptr);
    int rc = MBRWT_OK;
    auto cleanup = [&]() {
        for (auto &kv : tables) (void)hipFree(kv.second);
    };
    for (uint32_t u = 0; u < N && !rc; ++u) {
        const auto &sh = shape[u];
        if (sh.children.empty()) continue;
        std::vector<double> qc;
        for (uint32_t c : sh.children) qc.push_back(q[c]);
        auto it = tables.find(qc);
        if (it == tables.end()) {
            auto T = mask_table(qc);
            uint64_t *dT = nullptr;
            if (hipMalloc(&dT, T.size() * 8) != hipSuccess ||
                hipMemcpy(dT, T.data(), T.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
                rc = hip_fail(hipErrorOutOfMemory, "synthetic table upload");
                break;
            }
            it = tables.emplace(qc, dT).first;
        }
        node_T[u] = it->second;
    }
    if (rc) {
        cleanup();
        return rc;
    }
    unsigned long long *d_ones = nullptr;
    if (hipMalloc(&d_ones, sizeof(unsigned long long)) != hipSuccess) {
        cleanup();
        return hip_fail(hipErrorOutOfMemory, "hipMalloc");
    }
    (void)hipMemsetAsync(d_ones, 0, sizeof(unsigned long long), s);

    auto alloc_image = [&](DevNode &dn, uint64_t bytes) -> uint8_t * {
        void *p = nullptr;
        if (hipMalloc(&p, bytes + kImagePad) != hipSuccess) return nullptr;
        (void)hipMemsetAsync(p, 0, bytes + kImagePad, s);
        tree.images.push_back(p);
        tree.image_bytes += bytes + kImagePad;
        dn.base = (uint64_t)(uintptr_t)p;
        return reinterpret_cast<uint8_t *>(p);
    };
    auto fail = [&](int code, const char *what) {
        cleanup();
        (void)hipFree(d_ones);
        set_error(what);
        return code;
    };

    // super-root: the root's index column (Bernoulli(q_root) per row)
    {
        DevNode &sr = tree.nodes[0];
        sr.first_child = 1;
        sr.arity = 1;
        sr.label = UINT32_MAX;
        sr.length = n;
        const uint64_t K = root_key;
        const uint64_t T = prob_to_threshold(q[0]);
        if (shape[0].children.empty()) {  // one column: the root is a leaf
            sr.kind = KIND_MASK8;
            uint8_t *img = alloc_image(sr, n);
            if (!img) return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            hipLaunchKernelGGL(k_gen_root_mask, dim3(launch_grid(n)), dim3(256), 0, s, img, n, K, T, d_ones);
            if (hipGetLastError() != hipSuccess) return fail(MBRWT_ERR_DEVICE, "root mask kernel");
        } else {
            sr.kind = KIND_PLANE;
            sr.stride = 16;
            uint8_t *img = alloc_image(sr, ((n + 31) / 32) * sr.stride);
            if (!img) return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            hipLaunchKernelGGL(k_gen_root_plane, dim3(launch_grid((n + 31) / 32)), dim3(256), 0, s, img, n, K, T,
                               sr.stride);
            if (hipGetLastError() != hipSuccess) return fail(MBRWT_ERR_DEVICE, "root plane kernel");
            std::vector<uint64_t> tot;
            if ((rc = plane_scan(img, n, 1, sr.stride, tot, s))) return fail(rc, "root scan");
            // tot[0] = popcount of the root column = length of the root's children columns
            tree.nodes[1].length = tot[0];
            if (fold_root_enabled() && 2 * tot[0] >= n) {
                // fold the root into the super-root (mbrwt_internal.hpp): the
                // root plane above becomes a temporary input
                DevNode &rt = tree.nodes[1];
                const uint32_t a = rt.arity, nT = (1u << a) - 1;
                const bool plane = rt.kind == KIND_PLANE;
                void *tmp = tree.images.back();
                const uint64_t tmp_bytes = ((n + 31) / 32) * sr.stride + kImagePad;
                tree.images.pop_back();
                tree.image_bytes -= tmp_bytes;
                sr.kind = rt.kind;
                sr.arity = rt.arity;
                sr.stride = rt.stride;
                sr.first_child = rt.first_child;
                uint8_t *fimg = alloc_image(sr, plane ? ((n + 31) / 32) * sr.stride : n * mask_bytes(sr.kind));
                if (!fimg) {
                    (void)hipFree(tmp);
                    return fail(MBRWT_ERR_NOMEM, "device allocation failed");
                }
                fold_fn(a, plane)(fimg, n, reinterpret_cast<const uint8_t *>(tmp), keys[0], node_T[0],
                                  nT, sr.stride, d_ones, s);
                if (hipGetLastError() != hipSuccess) {
                    (void)hipFree(tmp);
                    return fail(MBRWT_ERR_DEVICE, "fold kernel");
                }
                if (plane) {
                    std::vector<uint64_t> ftot;
                    if ((rc = plane_scan(fimg, n, a, sr.stride, ftot, s))) {
                        (void)hipFree(tmp);
                        return fail(rc, "fold scan");
                    }
                    for (uint32_t c = 0; c < a; ++c) {
                        DevNode &ch = tree.nodes[shape[0].children[c] + 1];
                        if (ch.kind == KIND_LEAF) tree.num_relations += ftot[c];
                        else ch.length = ftot[c];
                    }
                }
                MBRWT_HIP(hipStreamSynchronize(s));
                (void)hipFree(tmp);
                rt.kind = KIND_FOLDED;
                rt.arity = 0;
                rt.first_child = 0;
                rt.base = 0;
                tree.folded = true;
            }
        }
    }
    // internal nodes in BFS order: parents are generated before children
    std::vector<bool> in_pack(N, false);  // MASK8 children of a KIND_PACK node, KIND_PACKT subtrees: no image
    unsigned long long *d_ctr = nullptr;
    if (hipMalloc(&d_ctr, 2 * sizeof(unsigned long long)) != hipSuccess) return fail(MBRWT_ERR_NOMEM, "hipMalloc");
    if (tree.folded && packt_enabled()) {
        if ((rc = synth_packt(shape, q, node_T, keys, tree, in_pack, d_ctr, d_ones, s))) {
            (void)hipFree(d_ctr);
            return fail(rc, "synthetic: KIND_PACKT generation");
        }
    }
    for (uint32_t u = 0; u < N; ++u) {
        const auto &sh = shape[u];
        DevNode &dn = tree.nodes[u + 1];
        if (sh.children.empty() || dn.kind == KIND_FOLDED || in_pack[u]) continue;
        const uint64_t L = dn.length;  // positions = popcount of u's own column
        const uint64_t K = keys[u];
        const uint32_t a = dn.arity, nT = (1u << a) - 1;
        // KIND_PACK2 when every child A is a PLANE node of <= 8 MASK8 children
        // with <= 8 leaves; span S = the largest of 8, 4, 2 at which a block
        // is expected to hold <= 56 bytes (S header bytes + S records; spills:
        // ~0.1 % of the blocks at the Kingsford shape, S = 8, mean 45.7 bytes;
        // a few % at the RefSeq shape, S = 2, mean 52.6 bytes)
        bool pack2 = pack2_enabled() && dn.kind == KIND_PLANE && a <= 8 && q[u] > 0.0;
        double rec = 1.0;
        std::vector<uint64_t *> utab;
        for (uint32_t c = 0; pack2 && c < a; ++c) {
            const uint32_t cu = sh.children[c];
            const DevNode &ch = tree.nodes[cu + 1];
            pack2 = ch.kind == KIND_PLANE && ch.arity <= 8;
            rec += q[cu] / q[u];
            for (uint32_t g = 0; pack2 && g < ch.arity; ++g) {
                const uint32_t gu = shape[cu].children[g];
                const DevNode &gn = tree.nodes[gu + 1];
                pack2 = gn.kind == KIND_MASK8 && gn.arity <= 8;
                rec += q[gu] / q[u];
                if (std::find(utab.begin(), utab.end(), node_T[gu]) == utab.end()) utab.push_back(node_T[gu]);
            }
        }
        uint32_t span = 0;
        for (uint32_t S = kPack2MaxSpan; pack2 && S >= 2 && !span; S /= 2)
            if (S * (rec + 1.0) <= 56.0) span = S;
        if (pack2 && (!span || utab.size() > 4)) pack2 = false;
        if (pack2) {
            std::vector<void *> tmps;
            auto free_tmps = [&]() {
                for (void *t : tmps) (void)hipFree(t);
            };
            auto tmp_plane = [&](uint64_t len, uint32_t stride) -> uint8_t * {
                void *t = nullptr;
                const uint64_t bytes = ((len + 31) / 32) * stride + kImagePad;
                if (hipMalloc(&t, bytes) != hipSuccess) return nullptr;
                (void)hipMemsetAsync(t, 0, bytes, s);
                tmps.push_back(t);
                return reinterpret_cast<uint8_t *>(t);
            };
            Pack2Args args{};
            args.a = a;
            args.ustride = dn.stride;
            uint8_t *up = tmp_plane(L, dn.stride);
            std::vector<uint64_t> tot;
            if (!up) {
                (void)hipFree(d_ctr);
                return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            }
            plane_fn(a)(up, L, K, node_T[u], nT, dn.stride, s);
            if ((rc = plane_scan(up, L, a, dn.stride, tot, s))) {
                free_tmps();
                (void)hipFree(d_ctr);
                return fail(rc, "plane scan");
            }
            args.uplane = up;
            for (uint32_t k = 0; k < utab.size(); ++k) {
                args.T[k] = utab[k];
                args.nT[k] = 255;
            }
            for (uint32_t c = 0; c < a; ++c) {
                const uint32_t cu = sh.children[c];
                DevNode &ch = tree.nodes[cu + 1];
                const uint32_t ca = ch.arity;
                ch.length = tot[c];
                uint8_t *ap = tmp_plane(tot[c], ch.stride);
                std::vector<uint64_t> gtot;
                if (!ap) {
                    free_tmps();
                    (void)hipFree(d_ctr);
                    return fail(MBRWT_ERR_NOMEM, "device allocation failed");
                }
                plane_fn(ca)(ap, tot[c], keys[cu], node_T[cu], (1u << ca) - 1, ch.stride, s);
                if ((rc = plane_scan(ap, tot[c], ca, ch.stride, gtot, s))) {
                    free_tmps();
                    (void)hipFree(d_ctr);
                    return fail(rc, "plane scan");
                }
                args.aplane[c] = ap;
                args.astride[c] = ch.stride;
                args.aarity[c] = ca;
                in_pack[cu] = true;
                ch.kind = KIND_PACK;  // record only (no image)
                ch.stride = kPackBlock;
                for (uint32_t g = 0; g < ca; ++g) {
                    const uint32_t gu = shape[cu].children[g];
                    DevNode &gn = tree.nodes[gu + 1];
                    gn.length = gtot[g];
                    gn.base = 0;
                    in_pack[gu] = true;
                    args.KB[8 * c + g] = keys[gu];
                    const uint32_t ti = (uint32_t)(std::find(utab.begin(), utab.end(), node_T[gu]) - utab.begin());
                    args.tB[8 * c + g] = (uint8_t)ti;
                    args.nT[ti] = (1u << gn.arity) - 1;
                }
            }
            const uint64_t nb2 = (L + span - 1) / span;
            (void)hipMemsetAsync(d_ctr, 0, 2 * sizeof(unsigned long long), s);
            hipLaunchKernelGGL(k_gen_pack2, dim3(launch_grid(nb2)), dim3(256), 0, s, nullptr, L, span, args, nullptr,
                               d_ctr, d_ones, 0);
            unsigned long long ctr2[2] = {0, 0};
            MBRWT_HIP(hipMemcpyAsync(ctr2, d_ctr, sizeof(ctr2), hipMemcpyDeviceToHost, s));
            MBRWT_HIP(hipStreamSynchronize(s));
            const unsigned long long spill_bytes = ctr2[0];
            if (ctr2[1]) {
                free_tmps();
                (void)hipFree(d_ctr);
                return fail(MBRWT_ERR_UNSUPPORTED, "synthetic: a PACK2 record longer than 64 bytes (density too high)");
            }
            uint8_t *spill = nullptr;
            if (spill_bytes) {
                DevNode dummy;
                spill = alloc_image(dummy, spill_bytes);
                if (!spill) {
                    free_tmps();
                    (void)hipFree(d_ctr);
                    return fail(MBRWT_ERR_NOMEM, "device allocation failed");
                }
            }
            dn.kind = KIND_PACK2;
            dn.stride = span;  // positions per block
            uint8_t *img = alloc_image(dn, nb2 * kPack2Block);
            if (!img) {
                free_tmps();
                (void)hipFree(d_ctr);
                return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            }
            (void)hipMemsetAsync(d_ctr, 0, sizeof(unsigned long long), s);
            hipLaunchKernelGGL(k_gen_pack2, dim3(launch_grid(nb2)), dim3(256), 0, s, img, L, span, args, spill, d_ctr,
                               d_ones, 1);
            if (hipGetLastError() != hipSuccess) {
                free_tmps();
                (void)hipFree(d_ctr);
                return fail(MBRWT_ERR_DEVICE, "pack2 kernel");
            }
            MBRWT_HIP(hipStreamSynchronize(s));
            free_tmps();
            continue;
        }
        // KIND_PACK when every child is a MASK8 node with <= 8 leaves and a
        // block of 16 positions is expected to hold <= 40 masks (spills: ~1 % of the blocks)
        bool pack = pack_enabled() && dn.kind == KIND_PLANE && a <= 8;
        double expect = 0.0;
        for (uint32_t c = 0; pack && c < a; ++c) {
            const DevNode &ch = tree.nodes[sh.children[c] + 1];
            pack = ch.kind == KIND_MASK8 && ch.arity <= 8;
            expect += q[sh.children[c]];
        }
        if (pack && q[u] > 0.0 && kPackSpan * expect / q[u] > 40.0) pack = false;
        if (pack) {
            void *tmp = nullptr;
            const uint64_t pbytes = ((L + 31) / 32) * dn.stride + kImagePad;
            if (hipMalloc(&tmp, pbytes) != hipSuccess) {
                (void)hipFree(d_ctr);
                return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            }
            (void)hipMemsetAsync(tmp, 0, pbytes, s);
            uint8_t *pl = reinterpret_cast<uint8_t *>(tmp);
            plane_fn(a)(pl, L, K, node_T[u], nT, dn.stride, s);
            std::vector<uint64_t> tot;
            if ((rc = plane_scan(pl, L, a, dn.stride, tot, s))) {
                (void)hipFree(tmp);
                (void)hipFree(d_ctr);
                return fail(rc, "plane scan");
            }
            PackArgs args{};
            for (uint32_t c = 0; c < a; ++c) {
                const uint32_t cu = sh.children[c];
                DevNode &ch = tree.nodes[cu + 1];
                ch.length = tot[c];
                ch.base = 0;
                in_pack[cu] = true;
                args.T[c] = node_T[cu];
                args.nT[c] = (1u << ch.arity) - 1;
                args.K[c] = keys[cu];
            }
            const uint32_t pstride = dn.stride;
            (void)hipMemsetAsync(d_ctr, 0, sizeof(unsigned long long), s);
            pack_fn(a)(nullptr, L, pl, pstride, args, nullptr, d_ctr, d_ones, 0, s);
            unsigned long long nspill = 0;
            MBRWT_HIP(hipMemcpyAsync(&nspill, d_ctr, sizeof(nspill), hipMemcpyDeviceToHost, s));
            MBRWT_HIP(hipStreamSynchronize(s));
            uint8_t *spill = nullptr;
            if (nspill) {
                DevNode dummy;
                spill = alloc_image(dummy, nspill * 128);
                if (!spill) {
                    (void)hipFree(tmp);
                    (void)hipFree(d_ctr);
                    return fail(MBRWT_ERR_NOMEM, "device allocation failed");
                }
            }
            dn.kind = KIND_PACK;
            dn.stride = kPackBlock;
            uint8_t *img = alloc_image(dn, ((L + kPackSpan - 1) / kPackSpan) * kPackBlock);
            if (!img) {
                (void)hipFree(tmp);
                (void)hipFree(d_ctr);
                return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            }
            (void)hipMemsetAsync(d_ctr, 0, sizeof(unsigned long long), s);
            pack_fn(a)(img, L, pl, pstride, args, spill, d_ctr, d_ones, 1, s);
            if (hipGetLastError() != hipSuccess) {
                (void)hipFree(tmp);
                (void)hipFree(d_ctr);
                return fail(MBRWT_ERR_DEVICE, "pack kernel");
            }
            MBRWT_HIP(hipStreamSynchronize(s));
            (void)hipFree(tmp);
            continue;
        }
        if (dn.kind == KIND_PLANE) {
            uint8_t *img = alloc_image(dn, ((L + 31) / 32) * dn.stride);
            if (!img) return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            plane_fn(a)(img, L, K, node_T[u], nT, dn.stride, s);
            if (hipGetLastError() != hipSuccess) return fail(MBRWT_ERR_DEVICE, "plane kernel");
            std::vector<uint64_t> tot;
            if ((rc = plane_scan(img, L, a, dn.stride, tot, s))) return fail(rc, "plane scan");
            for (uint32_t c = 0; c < a; ++c) {
                DevNode &ch = tree.nodes[sh.children[c] + 1];
                if (ch.kind == KIND_LEAF) tree.num_relations += tot[c];
                else ch.length = tot[c];
            }
        } else {
            uint8_t *img = alloc_image(dn, L * mask_bytes(dn.kind));
            if (!img) return fail(MBRWT_ERR_NOMEM, "device allocation failed");
            mask_fn(a)(img, L, K, node_T[u], nT, d_ones, s);
            if (hipGetLastError() != hipSuccess) return fail(MBRWT_ERR_DEVICE, "mask kernel");
        }
    }
    (void)hipFree(d_ctr);
    unsigned long long ones = 0;
    if (hipMemcpyAsync(&ones, d_ones, sizeof(ones), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return fail(MBRWT_ERR_DEVICE, "synthetic finish");
    tree.num_relations += ones;
    cleanup();
    (void)hipFree(d_ones);
    if (shard && shard->len_out) {  // positions of every internal node in this shard
        shard->len_out->assign(N, 0);
        for (uint32_t u = 0; u < N; ++u)
            if (!shape[u].children.empty()) (*shard->len_out)[u] = tree.nodes[u + 1].length;
    }
    return finalize_tree(tree);
}

}  // namespace mbrwt
