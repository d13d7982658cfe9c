// classify.hip -- StaticBinRelAnnotator::get_labels(indices, presence_ratio)
// (annotation/annotate_static.cpp:71-94) for a batch of reads on the device
// (SURVEY.md §8(f) row 2): the `classify` consumer of get_rows.
//
// One traversal for the rows of all reads (run_get_rows, CSR in workspaces),
// then one workgroup per read: the read's labels (a contiguous range of the
// CSR, its rows being contiguous) are counted in an LDS histogram
// (count_labels, annotate_static.cpp:149-162), and the labels present in at
// least ceil(|indices| * presence_ratio) rows (>= 1 row when the ratio is 0,
// :78-83) are written in ascending code order (:87-91).  Pass 0 counts them,
// a scan gives every read's output offset, pass 1 writes.
// get_top_labels(indices, num_top) (annotate.cpp:57-83; classify
// --count-labels, main.cpp:177) runs the same driver with a sorting kernel.
#include <hipcub/hipcub.hpp>

#include <cmath>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"

namespace mbrwt {
namespace {

constexpr uint32_t kClsThreads = 256;
constexpr uint32_t kClsMaxColumns = 15360;  // LDS histogram of u32 counters (60 KB)

__global__ __launch_bounds__(kClsThreads) void k_read_labels(const uint64_t *__restrict__ read_off, uint64_t n_reads,
                                                             uint64_t n_rows, const uint64_t *__restrict__ row_csr,
                                                             const uint32_t *__restrict__ cols, uint32_t m,
                                                             double ratio, uint64_t *__restrict__ counts_or_offsets,
                                                             uint32_t *__restrict__ out, int pass, uint64_t cap) {
    extern __shared__ uint32_t hist[];
    using Scan = hipcub::BlockScan<uint32_t, kClsThreads>;
    __shared__ typename Scan::TempStorage scan_tmp;
    const uint32_t t = threadIdx.x;
    const uint32_t per = (m + kClsThreads - 1) / kClsThreads;  // columns per thread, in order
    for (uint64_t r = blockIdx.x; r < n_reads; r += gridDim.x) {
        for (uint32_t i = t; i < m; i += kClsThreads) hist[i] = 0;
        __syncthreads();
        const uint64_t rs = gld(read_off + r), re = gld(read_off + r + 1);
        if (rs > re || re > n_rows || (r == 0 && rs != 0) || (r + 1 == n_reads && re != n_rows)) {
            // malformed read offsets: flag (pass 0 only runs over them) and skip
            if (t == 0) {
                gst(counts_or_offsets + r, (uint64_t)0);
                gst(counts_or_offsets + n_reads, (uint64_t)1);
            }
            __syncthreads();
            continue;
        }
        const uint64_t l0 = gld(row_csr + rs), l1 = gld(row_csr + re);
        for (uint64_t i = l0 + t; i < l1; i += kClsThreads) atomicAdd(&hist[gld(cols + i)], 1u);
        __syncthreads();
        // annotate_static.cpp:78-83 (same double arithmetic as the reference)
        const uint64_t len = re - rs;
        const uint64_t thr = ratio == 0.0 ? 1 : (uint64_t)std::ceil((double)len * ratio);
        uint32_t mine = 0;
        for (uint32_t k = 0; k < per; ++k) {
            const uint32_t col = t * per + k;
            if (col < m && hist[col] && hist[col] >= thr) ++mine;
        }
        uint32_t before, total;
        Scan(scan_tmp).ExclusiveSum(mine, before, total);
        if (pass == 0) {  // (cap: get_top_labels' num_top, counted by this pass at ratio 0)
            if (t == 0) gst(counts_or_offsets + r, std::min<uint64_t>(total, cap));
        } else {
            uint64_t o = gld(counts_or_offsets + r) + before;
            for (uint32_t k = 0; k < per; ++k) {
                const uint32_t col = t * per + k;
                if (col < m && hist[col] && hist[col] >= thr) gst(out + o++, col);
            }
        }
        __syncthreads();
    }
}

// MultiLabelEncoded::get_top_labels (annotate.cpp:57-83) per read: the
// read's histogram in LDS as u64, turned into sort keys (count << 14 |
// 16383 - label) that are gathered, in any order, into a compact buffer of
// kTopCompact entries; a bitonic sort of pow2 >= nonzero keys in descending
// order then gives labels by count descending and equal counts by label
// ascending (one of the orders the reference's unstable std::sort may
// produce).  A read with more nonzero labels than the buffer holds sorts
// the whole histogram (P = pow2 >= m keys, zeros last) in place.  The
// per-read output sizes min(nonzero, num_top) come from k_read_labels'
// counting pass at ratio 0 (a u32 histogram); this kernel is the writing pass.
constexpr uint32_t kTopLabelBits = 14;
constexpr uint32_t kTopLabelMask = (1u << kTopLabelBits) - 1;
constexpr uint32_t kTopMaxColumns = 8192;  // P * 8 bytes of LDS <= 64 KB
constexpr uint32_t kTopCompact = 4 * kClsThreads;  // + 4 KB of u32 keys

// descending bitonic sort of key[0..Q), Q a power of two, one block
__device__ inline void bitonic_desc(unsigned long long *key, uint32_t Q) {
    const uint32_t t = threadIdx.x;
    for (uint32_t k = 2; k <= Q; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t lj = (uint32_t)__builtin_ctz(j);  // j is a power of two: no division
            for (uint32_t p = t; p < Q / 2; p += kClsThreads) {
                const uint32_t i = ((p >> lj) << (lj + 1)) | (p & (j - 1)), l = i + j;
                const unsigned long long a = key[i], b = key[l];
                // runs with (i & k) == 0 descend, so the whole array ends descending
                if (((i & k) == 0) ? (a < b) : (a > b)) {
                    key[i] = b;
                    key[l] = a;
                }
            }
            __syncthreads();
        }
    }
}

// descending bitonic sort of u32 keys key[0..Q), Q a power of two in
// [4, 4 * kClsThreads], one block.  Thread t keeps keys 4t..4t+3 in
// registers: the j = 1, 2 steps of a merge are register compare-exchanges,
// the 4 <= j < 256 steps pair lanes of one wave (shuffles, no barrier), and
// only the j >= 256 steps go through LDS with block barriers.
__device__ inline void bitonic_desc_u32(uint32_t *key, uint32_t Q) {
    const uint32_t t = threadIdx.x;
    const bool own = 4 * t < Q;
    uint32_t v[4] = {0, 0, 0, 0};
    if (own) {
        const u32x4_t q = *reinterpret_cast<const u32x4_t *>(key + 4 * t);
        v[0] = q[0], v[1] = q[1], v[2] = q[2], v[3] = q[3];
    }
    auto reg_step = [&](uint32_t k, uint32_t j) {
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t l = r ^ j;
            if (l > r) {
                const bool desc = ((4 * t + r) & k) == 0;
                const uint32_t a = v[r], b = v[l];
                if (desc ? (a < b) : (a > b)) {
                    v[r] = b;
                    v[l] = a;
                }
            }
        }
    };
    // partner key e ^ j (j >= 4) sits in lane t ^ (j / 4), same register
    auto wave_step = [&](uint32_t k, uint32_t j) {
        const bool lower = ((4 * t) & j) == 0, desc = ((4 * t) & k) == 0;
        const bool keep_max = lower == desc;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t pv = (uint32_t)__shfl_xor((int)v[r], (int)(j >> 2), 64);
            v[r] = keep_max ? (v[r] > pv ? v[r] : pv) : (v[r] < pv ? v[r] : pv);
        }
    };
    for (uint32_t k = 2; k <= Q; k <<= 1) {
        uint32_t j = k >> 1;
        if (j >= 256) {
            if (own) *reinterpret_cast<u32x4_t *>(key + 4 * t) = u32x4_t{v[0], v[1], v[2], v[3]};
            __syncthreads();
            for (; j >= 256; j >>= 1) {
                const uint32_t lj = (uint32_t)__builtin_ctz(j);
                for (uint32_t p = t; p < Q / 2; p += kClsThreads) {
                    const uint32_t i = ((p >> lj) << (lj + 1)) | (p & (j - 1)), l = i + j;
                    const uint32_t a = key[i], b = key[l];
                    if (((i & k) == 0) ? (a < b) : (a > b)) {
                        key[i] = b;
                        key[l] = a;
                    }
                }
                __syncthreads();
            }
            if (own) {
                const u32x4_t q = *reinterpret_cast<const u32x4_t *>(key + 4 * t);
                v[0] = q[0], v[1] = q[1], v[2] = q[2], v[3] = q[3];
            }
        }
        for (; j >= 4; j >>= 1) wave_step(k, j);
        if (j == 2) reg_step(k, 2), j = 1;
        reg_step(k, 1);
    }
    if (own) *reinterpret_cast<u32x4_t *>(key + 4 * t) = u32x4_t{v[0], v[1], v[2], v[3]};
    __syncthreads();
}

__global__ __launch_bounds__(kClsThreads) void k_read_top_labels(const uint64_t *__restrict__ read_off,
                                                                 uint64_t n_reads, uint64_t n_rows,
                                                                 const uint64_t *__restrict__ row_csr,
                                                                 const uint32_t *__restrict__ cols, uint32_t m,
                                                                 uint32_t P, uint64_t num_top,
                                                                 const uint64_t *__restrict__ lab_off,
                                                                 uint32_t *__restrict__ out_labels,
                                                                 uint64_t *__restrict__ out_counts) {
    extern __shared__ unsigned long long key[];  // [P] histogram / keys, then u32 [kTopCompact]
    uint32_t *compact = reinterpret_cast<uint32_t *>(key + P);
    __shared__ uint32_t nz_all;
    const uint32_t t = threadIdx.x;
    for (uint64_t r = blockIdx.x; r < n_reads; r += gridDim.x) {
        for (uint32_t i = t; i < P; i += kClsThreads) key[i] = 0;
        if (t == 0) nz_all = 0;
        __syncthreads();
        const uint64_t rs = gld(read_off + r), re = gld(read_off + r + 1);
        // (the offsets were validated by the counting pass, k_read_labels)
        const uint64_t l0 = gld(row_csr + rs), l1 = gld(row_csr + re);
        for (uint64_t i = l0 + t; i < l1; i += kClsThreads) atomicAdd(&key[gld(cols + i)], 1ull);
        __syncthreads();
        // keys in place; the nonzero ones gathered with one LDS atomic per wave
        // (ballot + popcount; a per-label atomic on one counter serialises)
        const uint32_t lane = t & 63;
        for (uint32_t c = t; c < m; c += kClsThreads) {
            const unsigned long long k = key[c];
            const unsigned long long kk = (k << kTopLabelBits) | (kTopLabelMask - c);
            if (k) key[c] = kk;
            const uint64_t bal = __ballot(k != 0);
            if (bal) {
                const int leader = __ffsll((unsigned long long)bal) - 1;
                uint32_t b = 0;
                if ((int)lane == leader) b = atomicAdd(&nz_all, (uint32_t)__popcll(bal));
                b = (uint32_t)__shfl((int)b, leader, 64);
                const uint32_t at = b + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
                if (k && at < kTopCompact) compact[at] = (uint32_t)kk;  // used when count < 2^18
            }
        }
        __syncthreads();
        const uint32_t nz = nz_all;
        const uint64_t n_out = std::min<uint64_t>(nz, num_top);
        if (n_out) {
            const uint64_t o = gld(lab_off + r);
            // u32 keys (count < 2^18: a read of fewer than 2^18 rows) in the compact buffer
            if (nz <= kTopCompact && re - rs < (1ull << (32 - kTopLabelBits))) {
                uint32_t Q = 4;
                while (Q < nz) Q <<= 1;
                for (uint32_t i = nz + t; i < Q; i += kClsThreads) compact[i] = 0;
                __syncthreads();
                bitonic_desc_u32(compact, Q);
                for (uint32_t i = t; i < n_out; i += kClsThreads) {
                    const uint32_t k = compact[i];
                    gst(out_labels + o + i, kTopLabelMask - (k & kTopLabelMask));
                    gst(out_counts + o + i, (uint64_t)(k >> kTopLabelBits));
                }
            } else {
                bitonic_desc(key, P);
                for (uint32_t i = t; i < n_out; i += kClsThreads) {
                    const unsigned long long k = key[i];
                    gst(out_labels + o + i, kTopLabelMask - (uint32_t)(k & kTopLabelMask));
                    gst(out_counts + o + i, (uint64_t)(k >> kTopLabelBits));
                }
            }
        }
        __syncthreads();
    }
}

unsigned grid_of(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(n, 65536)); }

}  // namespace

// The rows of all reads through the scheme's get_rows (CSR in io.off /
// io.cols, grown on MBRWT_ERR_CAPACITY), then launch(pass 0, counts) per
// read, a scan into d_lab_off, the capacity check and launch(pass 1,
// d_lab_off).  Shared by get_labels and get_top_labels of both schemes.
template <class Launch>
int classify_batch(const ClassifyIo &io, const ClassifyRowsFn &get_rows, uint64_t n_rows, uint64_t n_reads,
                   uint64_t *d_lab_off, bool have_out, uint64_t cap, uint64_t *needed, hipStream_t s, Launch launch) {
    if (!n_reads && n_rows) {  // the one offset would have to be both 0 and n_rows
        set_error("read offsets must ascend from 0 to n_rows");
        return MBRWT_ERR_INVALID;
    }
    if (n_reads > 0x7FFFFFF0ull) {  // hipCUB scans take int item counts
        set_error("batch larger than 2^31 reads");
        return MBRWT_ERR_UNSUPPORTED;
    }
    int rc;
    // 1. the labels of every row of every read
    if ((rc = ensure(*io.off, (n_rows + 1) * sizeof(uint64_t)))) return rc;
    uint64_t *d_off = reinterpret_cast<uint64_t *>(io.off->buf);
    uint64_t need = 0;
    rc = get_rows(d_off, reinterpret_cast<uint32_t *>(io.cols->buf), io.cols->bytes / sizeof(uint32_t), &need);
    if (rc == MBRWT_ERR_CAPACITY) {
        if ((rc = ensure(*io.cols, (need + need / 8 + 1024) * sizeof(uint32_t)))) return rc;
        rc = get_rows(d_off, reinterpret_cast<uint32_t *>(io.cols->buf), io.cols->bytes / sizeof(uint32_t), &need);
    }
    if (rc) return rc;
    if (!n_reads) {
        MBRWT_HIP(hipMemsetAsync(d_lab_off, 0, sizeof(uint64_t), s));
        MBRWT_HIP(hipStreamSynchronize(s));
        if (needed) *needed = 0;
        return MBRWT_OK;
    }
    const uint32_t *d_cols = reinterpret_cast<const uint32_t *>(io.cols->buf);
    // 2. per-read counts, inclusive scan -> d_lab_off[1..n_reads]
    //    (d_cnt[n_reads] = the malformed-offsets flag)
    if ((rc = ensure(*io.cnt, (n_reads + 1) * sizeof(uint64_t)))) return rc;
    uint64_t *d_cnt = reinterpret_cast<uint64_t *>(io.cnt->buf);
    MBRWT_HIP(hipMemsetAsync(d_cnt + n_reads, 0, sizeof(uint64_t), s));
    launch(0, d_off, d_cols, d_cnt);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemsetAsync(d_lab_off, 0, sizeof(uint64_t), s));
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, d_cnt, d_lab_off + 1, (int)n_reads, s));
    if ((rc = ensure(*io.scan, scan_bytes + 16))) return rc;
    MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(io.scan->buf, scan_bytes, d_cnt, d_lab_off + 1, (int)n_reads, s));
    uint64_t total = 0, bad = 0;
    MBRWT_HIP(hipMemcpyAsync(&total, d_lab_off + n_reads, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipMemcpyAsync(&bad, d_cnt + n_reads, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (bad) {
        set_error("read offsets must ascend from 0 to n_rows");
        return MBRWT_ERR_INVALID;
    }
    if (needed) *needed = total;
    if (total > cap || (total && !have_out)) {
        set_error("label buffer too small (see labels_needed)");
        return MBRWT_ERR_CAPACITY;
    }
    // 3. the output
    if (total) {
        launch(1, d_off, d_cols, d_lab_off);
        MBRWT_HIP(hipGetLastError());
    }
    return MBRWT_OK;
}

int classify_labels(const ClassifyIo &io, const ClassifyRowsFn &get_rows, uint64_t m, uint64_t n_rows,
                    const uint64_t *d_read_off, uint64_t n_reads, double ratio, uint64_t *d_lab_off, uint32_t *d_labels,
                    uint64_t cap, uint64_t *needed, hipStream_t s) {
    if (!(ratio >= 0.0 && ratio <= 1.0)) {  // an assert in the reference (annotate_static.cpp:76)
        set_error("presence_ratio outside [0, 1]");
        return MBRWT_ERR_INVALID;
    }
    if (m > kClsMaxColumns) {
        set_error("get_labels batch: more than 15360 columns is not supported by this build");
        return MBRWT_ERR_UNSUPPORTED;
    }
    const size_t lds = std::max<uint64_t>(m, 1) * sizeof(uint32_t);
    return classify_batch(io, get_rows, n_rows, n_reads, d_lab_off, d_labels != nullptr, cap, needed, s,
                          [&](int pass, const uint64_t *d_off, const uint32_t *d_cols, uint64_t *cnt_or_off) {
                              hipLaunchKernelGGL(k_read_labels, dim3(grid_of(n_reads)), dim3(kClsThreads), lds, s,
                                                 d_read_off, n_reads, n_rows, d_off, d_cols, (uint32_t)m, ratio,
                                                 cnt_or_off, pass ? d_labels : nullptr, pass, ~0ull);
                          });
}

int classify_top_labels(const ClassifyIo &io, const ClassifyRowsFn &get_rows, uint64_t m, uint64_t n_rows,
                        const uint64_t *d_read_off, uint64_t n_reads, uint64_t num_top, uint64_t *d_lab_off,
                        uint32_t *d_labels, uint64_t *d_counts, uint64_t cap, uint64_t *needed, hipStream_t s) {
    if (m > kTopMaxColumns) {
        set_error("get_top_labels batch: more than 8192 columns is not supported by this build");
        return MBRWT_ERR_UNSUPPORTED;
    }
    uint32_t P = 2;
    while (P < m) P <<= 1;
    const size_t lds = (size_t)P * sizeof(unsigned long long) + kTopCompact * sizeof(uint32_t);
    return classify_batch(io, get_rows, n_rows, n_reads, d_lab_off, d_labels && d_counts, cap, needed, s,
                          [&](int pass, const uint64_t *d_off, const uint32_t *d_cols, uint64_t *cnt_or_off) {
                              if (pass == 0) {  // min(distinct labels, num_top): a u32 histogram suffices
                                  hipLaunchKernelGGL(k_read_labels, dim3(grid_of(n_reads)), dim3(kClsThreads),
                                                     std::max<uint64_t>(m, 1) * sizeof(uint32_t), s, d_read_off,
                                                     n_reads, n_rows, d_off, d_cols, (uint32_t)m, 0.0, cnt_or_off,
                                                     nullptr, 0, num_top);
                                  return;
                              }
                              hipLaunchKernelGGL(k_read_top_labels, dim3(grid_of(n_reads)), dim3(kClsThreads), lds,
                                                 s, d_read_off, n_reads, n_rows, d_off, d_cols, (uint32_t)m, P,
                                                 num_top, cnt_or_off, d_labels, d_counts);
                          });
}

namespace {
ClassifyIo brwt_io(Ctx &c) { return ClassifyIo{&c.ws_cls_off, &c.ws_cls_cols, &c.ws_sort, &c.ws_scan}; }
}  // namespace

int run_get_labels_batch(Ctx &c, const uint64_t *d_rows, uint64_t n_rows, const uint64_t *d_read_off, uint64_t n_reads,
                         double ratio, uint64_t *d_lab_off, uint32_t *d_labels, uint64_t cap, uint64_t *needed,
                         hipStream_t s) {
    const ClassifyRowsFn rows = [&](uint64_t *d_off, uint32_t *d_cols, uint64_t cols_cap, uint64_t *need) {
        return run_get_rows(c, d_rows, n_rows, d_off, d_cols, cols_cap, need, s);
    };
    return classify_labels(brwt_io(c), rows, c.tree.num_columns, n_rows, d_read_off, n_reads, ratio, d_lab_off,
                           d_labels, cap, needed, s);
}

int run_get_top_labels_batch(Ctx &c, const uint64_t *d_rows, uint64_t n_rows, const uint64_t *d_read_off,
                             uint64_t n_reads, uint64_t num_top, uint64_t *d_lab_off, uint32_t *d_labels,
                             uint64_t *d_counts, uint64_t cap, uint64_t *needed, hipStream_t s) {
    const ClassifyRowsFn rows = [&](uint64_t *d_off, uint32_t *d_cols, uint64_t cols_cap, uint64_t *need) {
        return run_get_rows(c, d_rows, n_rows, d_off, d_cols, cols_cap, need, s);
    };
    return classify_top_labels(brwt_io(c), rows, c.tree.num_columns, n_rows, d_read_off, n_reads, num_top, d_lab_off,
                               d_labels, d_counts, cap, needed, s);
}

}  // namespace mbrwt
