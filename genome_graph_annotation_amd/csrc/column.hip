// column.hip -- column query BRWT::get_column (BRWT.cpp:55-85) on the device.
//
// The reference walks down to the leaf holding the column and lifts the
// leaf's set positions back up: at every internal node, child-local row i
// becomes parent row select1(i + 1) of the node's index column
// (bit_vector_rrr::select1, bit_vector.cpp:863-869; 1-based).  Here:
//   1. the leaf's set positions are read out of its parent's image (bit c of
//      the MASK words, or of the PLANE block words) with a two-pass stream
//      compaction (per-block counts -> scan -> ordered write),
//   2. each ancestor's select1 is a binary search over the per-32-position
//      rank words of that node's column inside ITS parent's interleaved
//      image, followed by a select inside one 32-bit word.
// Positions stay ascending through every lift (select1 is monotone), so the
// result is the reference's ascending row list.
#include <hipcub/hipcub.hpp>

#include <vector>

#include "device_access.hpp"
#include "mbrwt_internal.hpp"
#include "pack_block.hpp"

namespace mbrwt {
namespace {

constexpr int kColThreads = 256;  // one thread = one 32-position word

// Word w (positions 32w .. 32w+31, clipped to len) of child slot c's column
// inside the image of node nd.  For a KIND_PACK node the word marks the
// positions where child c is set AND its MASK8 mask has bit `leaf` (the
// leaf's positions lifted through the image-less MASK8 child at once); for a
// KIND_PACK2 node, where child c, its child leaf >> 8 and that child's leaf
// (leaf & 0xFF) are all set (two image-less levels lifted at once).
// For a KIND_PACKT node (dnode v) the word marks the positions whose record
// holds the leaf with pre-order label `leaf`.
__device__ __forceinline__ uint32_t column_word(const DevNode *nodes, uint32_t v, const DevNode &nd, uint32_t c,
                                                uint64_t w, uint64_t len, uint32_t leaf) {
    if (32 * w >= len) return 0;
    uint32_t bits = 0;
    if (nd.kind == KIND_PACKT) {
        const uint32_t S = nd.stride;  // positions per block (any of 1..8)
        Pack2Block pb;
        uint64_t cur = ~0ull;
        for (uint32_t h = 0; h < 32; ++h) {
            const uint64_t j = 32 * w + h;
            if (j >= len) break;
            if (j / S != cur) {
                cur = j / S;
                pb.load(nd.base, (uint32_t)j, S);
            }
            uint32_t hit = 0;
            (void)packt_walk(
                nodes, v, [&](uint32_t o) { return pb.byte(o); }, pb.start((uint32_t)(j % S)),
                [&](uint32_t label) { hit |= label == leaf; }, [](uint32_t) {});
            bits |= hit << h;
        }
    } else if (nd.kind == KIND_PACK2) {  // leaf = (B << 8) | leaf slot of the MASK8 grandchild B below child c
        const uint32_t B = leaf >> 8, lf = leaf & 0xFFu;
        const uint32_t S = nd.stride;  // positions per block
        for (uint32_t h = 0; h < 32; h += S) {
            const uint64_t j0 = 32 * w + h;
            if (j0 >= len) break;
            Pack2Block pb;
            pb.load(nd.base, (uint32_t)j0, S);
            for (uint32_t t = 0; t < S && j0 + t < len; ++t) {
                const uint32_t s = pb.start(t);
                const uint32_t m2 = pb.byte(s);
                if (!((m2 >> c) & 1u)) continue;
                const uint32_t i = (uint32_t)__builtin_popcount(m2 & ((1u << c) - 1u));
                const uint32_t m1 = pb.byte(s + 1 + i);
                if (!((m1 >> B) & 1u)) continue;
                uint32_t o = s + 1 + (uint32_t)__builtin_popcount(m2);
                for (uint32_t q = 0; q < i; ++q) o += (uint32_t)__builtin_popcount(pb.byte(s + 1 + q));
                o += (uint32_t)__builtin_popcount(m1 & ((1u << B) - 1u));
                if ((pb.byte(o) >> lf) & 1u) bits |= 1u << (h + t);
            }
        }
    } else if (nd.kind == KIND_PACK) {
        for (uint32_t h = 0; h < 32 / kPackSpan; ++h) {
            const uint64_t j0 = 32 * w + kPackSpan * h;
            if (j0 >= len) break;
            PackBlock pb;
            pb.load(nd.base, (uint32_t)j0);
            uint32_t o = 0;
            for (uint32_t q = 0; q < c; ++q) o += (uint32_t)__builtin_popcount(pb.bits(q));
            uint32_t bc = pb.bits(c);
            for (uint32_t x = bc; x; x &= x - 1) {
                const uint32_t t = (uint32_t)__builtin_ctz(x);
                const uint32_t m = pb.mask(o + (uint32_t)__builtin_popcount(bc & ((1u << t) - 1u)));
                if ((m >> leaf) & 1u) bits |= 1u << (kPackSpan * h + t);
            }
        }
    } else if (nd.kind == KIND_PLANE) {
        bits = gld_at<uint32_t>(nd.base + w * nd.stride + 8u * c + 4u);
    } else {
        const uint32_t W = 1u << (nd.kind - KIND_MASK8);
        const uint64_t end = len - 32 * w < 32 ? len - 32 * w : 32;
        for (uint32_t k = 0; k < end; ++k) {
            const uint64_t addr = nd.base + (32 * w + k) * W;
            uint64_t m;
            if (W == 1) m = gld_at<uint8_t>(addr);
            else if (W == 2) m = gld_at<uint16_t>(addr);
            else if (W == 4) m = gld_at<uint32_t>(addr);
            else m = gld_at<uint64_t>(addr);
            bits |= (uint32_t)((m >> c) & 1u) << k;
        }
    }
    const uint64_t rem = len - 32 * w;
    if (rem < 32) bits &= (1u << rem) - 1u;
    return bits;
}

__global__ __launch_bounds__(kColThreads) void k_col_count(const DevNode *nodes, uint32_t v, DevNode nd, uint32_t c,
                                                           uint32_t leaf, uint64_t len, uint64_t nwords,
                                                           uint64_t *block_counts) {
    using Reduce = hipcub::BlockReduce<uint32_t, kColThreads>;
    __shared__ typename Reduce::TempStorage tmp;
    const uint64_t w = (uint64_t)blockIdx.x * kColThreads + threadIdx.x;
    const uint32_t n = w < nwords ? (uint32_t)__builtin_popcount(column_word(nodes, v, nd, c, w, len, leaf)) : 0u;
    const uint32_t total = Reduce(tmp).Sum(n);
    if (threadIdx.x == 0) block_counts[blockIdx.x] = total;
}

__global__ __launch_bounds__(kColThreads) void k_col_write(const DevNode *nodes, uint32_t v, DevNode nd, uint32_t c,
                                                           uint32_t leaf, uint64_t len, uint64_t nwords,
                                                           const uint64_t *block_offsets, uint32_t *out) {
    using Scan = hipcub::BlockScan<uint32_t, kColThreads>;
    __shared__ typename Scan::TempStorage tmp;
    const uint64_t w = (uint64_t)blockIdx.x * kColThreads + threadIdx.x;
    uint32_t bits = w < nwords ? column_word(nodes, v, nd, c, w, len, leaf) : 0u;
    uint32_t pre;
    Scan(tmp).ExclusiveSum((uint32_t)__builtin_popcount(bits), pre);
    uint64_t o = block_offsets[blockIdx.x] + pre;
    while (bits) {
        out[o++] = (uint32_t)(32 * w) + (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1;
    }
}

// positions in the child's space -> positions in the parent's space:
// pos = select1(column c of nd's image, pos + 1)
__global__ __launch_bounds__(256) void k_col_lift(DevNode nd, uint32_t c, uint64_t nblocks, uint32_t *pos,
                                                  uint64_t n) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) {
        const uint32_t k = pos[i] + 1;  // 1-based rank of the wanted one
        // last block whose rank-before is < k (block 0 has rank 0)
        uint64_t lo = 0, hi = nblocks;
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (gld_at<uint32_t>(nd.base + mid * nd.stride + 8u * c) < k) lo = mid;
            else hi = mid;
        }
        const uint2 rb = gld_at<uint2>(nd.base + lo * nd.stride + 8u * c);
        uint32_t bits = rb.y;
        for (uint32_t r = k - rb.x; r > 1; --r) bits &= bits - 1;  // drop the r-1 lowest ones
        pos[i] = (uint32_t)(32 * lo) + (uint32_t)__builtin_ctz(bits);
    }
}

__global__ void k_widen(const uint32_t *in, uint64_t *out, uint64_t n) {
    const uint64_t gstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gstride) out[i] = in[i];
}

unsigned grid_of(uint64_t n, unsigned per) {
    const uint64_t g = (n + per - 1) / per;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 65535 * 16));
}

}  // namespace

int run_get_column(Ctx &c, uint64_t column, uint64_t *d_rows, uint64_t rows_cap, uint64_t *rows_needed,
                   hipStream_t s) {
    if (c.nodes_freed) return rows_get_column(c, column, d_rows, rows_cap, rows_needed, s);
    if (!c.shards.empty()) return sharded_get_column(c, column, d_rows, rows_cap, rows_needed, s);
    const Tree &t = c.tree;
    if (column >= t.num_columns) {
        set_error("column out of range");
        return MBRWT_ERR_RANGE;
    }
    // the path (dnode, child slot) from the super-root down to the leaf's parent
    std::vector<std::pair<uint32_t, uint32_t>> path;
    uint32_t v = 0;
    for (uint32_t k = 0; k < t.path_len; ++k) {
        const uint32_t slot = t.col_path[column * t.path_len + k];
        path.emplace_back(v, slot);
        const uint32_t w = t.nodes[v].first_child + slot;
        if (t.nodes[w].kind == KIND_LEAF) break;
        v = w;
    }
    if (path.empty() || t.nodes[t.nodes[path.back().first].first_child + path.back().second].kind != KIND_LEAF) {
        set_error("inconsistent column path");
        return MBRWT_ERR_INVALID;
    }
    // the leaf's positions come out of its parent's image -- or, when that
    // parent is a MASK8 child of a KIND_PACK node, out of the PACK image
    // (positions in the PACK node's space; the MASK8 level has no image)
    uint32_t leaf_bit = 0;
    size_t pt = 0;
    while (pt < path.size() && t.nodes[path[pt].first].kind != KIND_PACKT) ++pt;
    if (pt < path.size()) {
        // a KIND_PACKT ancestor: positions come out of its records (the
        // levels below it have no image); leaf_bit = the leaf's pre-order label
        leaf_bit = t.nodes[t.col_leaf[column]].label;
        path.resize(pt + 1);
    } else if (path.size() >= 3 && t.nodes[path[path.size() - 3].first].kind == KIND_PACK2) {
        // two image-less levels: positions come out of the PACK2 node's records
        leaf_bit = path.back().second;
        path.pop_back();
        leaf_bit |= path.back().second << 8;
        path.pop_back();
    } else if (path.size() >= 2 && t.nodes[path[path.size() - 2].first].kind == KIND_PACK) {
        leaf_bit = path.back().second;
        path.pop_back();
    }
    const uint32_t leaf_parent_id = path.back().first;
    const DevNode leaf_parent = t.nodes[leaf_parent_id];
    const uint32_t leaf_slot = path.back().second;
    const uint64_t len = leaf_parent.length;
    const uint64_t nwords = (len + 31) / 32;
    const uint64_t nblk = std::max<uint64_t>(1, (nwords + kColThreads - 1) / kColThreads);

    int rc;
    size_t scan_bytes = 0;
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                               (int)nblk, s));
    if ((rc = ensure(c.ws_counts, 2 * (nblk + 1) * sizeof(uint64_t)))) return rc;
    c.rows_sc_dirty = true;  // (the row-record kernels' counters live in ws_counts)
    if ((rc = ensure(c.ws_scan, scan_bytes + 16))) return rc;
    uint64_t *d_cnt = reinterpret_cast<uint64_t *>(c.ws_counts.buf);
    uint64_t *d_off = d_cnt + nblk + 1;
    if (nwords) {
        hipLaunchKernelGGL(k_col_count, dim3((unsigned)nblk), dim3(kColThreads), 0, s, (const DevNode *)c.d_nodes,
                           leaf_parent_id, leaf_parent, leaf_slot, leaf_bit,
                           len, nwords, d_cnt);
        MBRWT_HIP(hipGetLastError());
    } else {
        MBRWT_HIP(hipMemsetAsync(d_cnt, 0, nblk * sizeof(uint64_t), s));
    }
    MBRWT_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_scan.buf, scan_bytes, d_cnt, d_off, (int)nblk, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars, d_off + nblk - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipMemcpyAsync(c.h_scalars + 1, d_cnt + nblk - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MBRWT_HIP(hipStreamSynchronize(s));
    const uint64_t total = c.h_scalars[0] + c.h_scalars[1];
    if (rows_needed) *rows_needed = total;
    if (total > rows_cap || (total && !d_rows)) {
        set_error("row buffer too small (see rows_needed)");
        return MBRWT_ERR_CAPACITY;
    }
    if (!total) return MBRWT_OK;

    if ((rc = ensure(c.ws_temp, total * sizeof(uint32_t)))) return rc;
    uint32_t *d_pos = reinterpret_cast<uint32_t *>(c.ws_temp.buf);
    hipLaunchKernelGGL(k_col_write, dim3((unsigned)nblk), dim3(kColThreads), 0, s, (const DevNode *)c.d_nodes,
                       leaf_parent_id, leaf_parent, leaf_slot, leaf_bit,
                       len, nwords, d_off, d_pos);
    MBRWT_HIP(hipGetLastError());
    // lift through the ancestors: node path[k+1].first's column lives in the
    // image of path[k].first at slot path[k].second
    for (size_t k = path.size() - 1; k-- > 0;) {
        const DevNode nd = t.nodes[path[k].first];
        const uint64_t nb = (nd.length + 31) / 32;
        hipLaunchKernelGGL(k_col_lift, dim3(grid_of(total, 256)), dim3(256), 0, s, nd, path[k].second, nb, d_pos,
                           total);
        MBRWT_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_widen, dim3(grid_of(total, 256)), dim3(256), 0, s, d_pos, d_rows, total);
    MBRWT_HIP(hipGetLastError());
    return MBRWT_OK;
}

}  // namespace mbrwt
