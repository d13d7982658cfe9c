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
                                                             uint32_t *__restrict__ out, int pass) {
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
        if (pass == 0) {
            if (t == 0) gst(counts_or_offsets + r, (uint64_t)total);
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

unsigned grid_of(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(n, 65536)); }

}  // namespace

int run_get_labels_batch(Ctx &c, const uint64_t *d_rows, uint64_t n_rows, const uint64_t *d_read_off, uint64_t n_reads,
                         double ratio, uint64_t *d_lab_off, uint32_t *d_labels, uint64_t cap, uint64_t *needed,
                         hipStream_t s) {
    const uint64_t m = c.tree.num_columns;
    if (!(ratio >= 0.0 && ratio <= 1.0)) {  // an assert in the reference (annotate_static.cpp:76)
        set_error("presence_ratio outside [0, 1]");
        return MBRWT_ERR_INVALID;
    }
    if (m > kClsMaxColumns) {
        set_error("get_labels batch: more than 15360 columns is not supported by this build");
        return MBRWT_ERR_UNSUPPORTED;
    }
    if (!n_reads && n_rows) {  // the one offset would have to be both 0 and n_rows
        set_error("read offsets must ascend from 0 to n_rows");
        return MBRWT_ERR_INVALID;
    }
    int rc;
    // 1. the labels of every row of every read
    if ((rc = ensure(c.ws_cls_off, (n_rows + 1) * sizeof(uint64_t)))) return rc;
    uint64_t *d_off = reinterpret_cast<uint64_t *>(c.ws_cls_off.buf);
    uint64_t need = 0;
    rc = run_get_rows(c, d_rows, n_rows, d_off, reinterpret_cast<uint32_t *>(c.ws_cls_cols.buf),
                      c.ws_cls_cols.bytes / sizeof(uint32_t), &need, s);
    if (rc == MBRWT_ERR_CAPACITY) {
        if ((rc = ensure(c.ws_cls_cols, (need + need / 8 + 1024) * sizeof(uint32_t)))) return rc;
        rc = run_get_rows(c, d_rows, n_rows, d_off, reinterpret_cast<uint32_t *>(c.ws_cls_cols.buf),
                          c.ws_cls_cols.bytes / sizeof(uint32_t), &need, s);
    }
    if (rc) return rc;
    if (!n_reads) {
        MBRWT_HIP(hipMemsetAsync(d_lab_off, 0, sizeof(uint64_t), s));
        MBRWT_HIP(hipStreamSynchronize(s));
        if (needed) *needed = 0;
        return MBRWT_OK;
    }
    const uint32_t *d_cols = reinterpret_cast<const uint32_t *>(c.ws_cls_cols.buf);
    const size_t lds = std::max<uint64_t>(m, 1) * sizeof(uint32_t);
    // 2. per-read counts, inclusive scan -> d_lab_off[1..n_reads]
    //    (d_cnt[n_reads] = the malformed-offsets flag)
    if ((rc = ensure(c.ws_sort, (n_reads + 1) * sizeof(uint64_t)))) return rc;
    uint64_t *d_cnt = reinterpret_cast<uint64_t *>(c.ws_sort.buf);
    MBRWT_HIP(hipMemsetAsync(d_cnt + n_reads, 0, sizeof(uint64_t), s));
    hipLaunchKernelGGL(k_read_labels, dim3(grid_of(n_reads)), dim3(kClsThreads), lds, s, d_read_off, n_reads, n_rows,
                       d_off, d_cols, (uint32_t)m, ratio, d_cnt, nullptr, 0);
    MBRWT_HIP(hipGetLastError());
    MBRWT_HIP(hipMemsetAsync(d_lab_off, 0, sizeof(uint64_t), s));
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, d_cnt, d_lab_off + 1, (int)n_reads, s));
    if ((rc = ensure(c.ws_scan, scan_bytes + 16))) return rc;
    MBRWT_HIP(hipcub::DeviceScan::InclusiveSum(c.ws_scan.buf, scan_bytes, d_cnt, d_lab_off + 1, (int)n_reads, s));
    uint64_t total = 0, bad = 0;
    MBRWT_HIP(hipMemcpyAsync(&total, d_lab_off + n_reads, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipMemcpyAsync(&bad, d_cnt + n_reads, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    if (bad) {
        set_error("read offsets must ascend from 0 to n_rows");
        return MBRWT_ERR_INVALID;
    }
    if (needed) *needed = total;
    if (total > cap || (total && !d_labels)) {
        set_error("label buffer too small (see labels_needed)");
        return MBRWT_ERR_CAPACITY;
    }
    // 3. the labels, ascending per read
    if (total) {
        hipLaunchKernelGGL(k_read_labels, dim3(grid_of(n_reads)), dim3(kClsThreads), lds, s, d_read_off, n_reads,
                           n_rows, d_off, d_cols, (uint32_t)m, ratio, d_lab_off, d_labels, 1);
        MBRWT_HIP(hipGetLastError());
    }
    return MBRWT_OK;
}

}  // namespace mbrwt
