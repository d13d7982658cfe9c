// sdsl_format.hpp -- the byte formats of the reference's on-disk structures
// (header-only host C++; used by libmbrwt's BRWT reader/writer, brwt_io.cpp,
// and by the C++ mirror's LabelEncoder, annotate_static.hpp).
//
// The reference serialises through two third-party libraries that are absent
// from /root/reference (empty submodules):
//   * libmaus2 (akahles fork, branch `shrunk`): NumberSerialisation /
//     StringSerialisation -- call sites common/serialization.cpp:27-36,
//     common/annotate.cpp:33-52;
//   * sdsl-lite (hmusta fork): int_vector<> / bit_vector / rrr_vector<63>
//     serialisation -- call sites common/serialization.cpp:38-97 and
//     common/bit_vector.cpp:906-925.
// What follows restates their PUBLISHED algorithms: a libmaus2 number is 8
// bytes, most significant first; a string is its length (a number) then its
// bytes; an sdsl int_vector<> is {u64 size in bits, u8 width, ceil(size/64)
// little-endian u64 words}, a bit_vector the same without the width byte; an
// rrr_vector<63, int_vector<>, 32> is {u64 size, int_vector<> bt (block
// classes, width 6), bit_vector btnr (the blocks' combinatorial numbers,
// ceil(log2 C(63, class)) bits each), int_vector<> btnrp and rank (samples
// every 32 blocks), bit_vector invert (superblocks stored complemented)}.
// PARITY UNPINNED: no sdsl / libmaus2 source or reference-written file exists
// here, so these bytes are checked only by round trips and by the logical
// results (rank/select/access) of what is read back.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace mbrwt {
namespace fmt {

struct FormatError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ---- byte streams --------------------------------------------------------
struct Writer {
    std::vector<uint8_t> buf;
    void bytes(const void *p, size_t n) {
        const uint8_t *b = static_cast<const uint8_t *>(p);
        buf.insert(buf.end(), b, b + n);
    }
    void u8(uint8_t v) { buf.push_back(v); }
    void u64le(uint64_t v) {
        for (int i = 0; i < 8; ++i) buf.push_back((uint8_t)(v >> (8 * i)));
    }
};

struct Reader {
    const uint8_t *p;
    uint64_t n, pos = 0;
    Reader(const uint8_t *data, uint64_t len) : p(data), n(len) {}
    void need(uint64_t k) const {
        if (k > n - pos) throw FormatError("unexpected end of stream");
    }
    // words of 64 bits for `bits` bits, checked against the rest of the stream
    // BEFORE anything is sized from the (untrusted) header
    uint64_t words_for(uint64_t bits) const {
        const uint64_t W = bits / 64 + (bits % 64 != 0);
        if (W > (n - pos) / 8) throw FormatError("vector longer than the stream");
        return W;
    }
    uint8_t u8() {
        need(1);
        return p[pos++];
    }
    uint64_t u64le() {
        need(8);
        uint64_t v = 0;
        for (int i = 0; i < 8; ++i) v |= (uint64_t)p[pos + i] << (8 * i);
        pos += 8;
        return v;
    }
    void bytes(void *dst, uint64_t k) {
        need(k);
        std::memcpy(dst, p + pos, k);
        pos += k;
    }
};

// ---- libmaus2 NumberSerialisation / StringSerialisation ------------------
inline void put_number(Writer &w, uint64_t v) {  // serialiseNumber: 8 bytes, MSB first
    for (int i = 7; i >= 0; --i) w.u8((uint8_t)(v >> (8 * i)));
}
inline uint64_t get_number(Reader &r) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | r.u8();
    return v;
}
inline void put_string(Writer &w, const std::string &s) {
    put_number(w, s.size());
    w.bytes(s.data(), s.size());
}
inline std::string get_string(Reader &r) {
    const uint64_t len = get_number(r);
    r.need(len);
    std::string s(reinterpret_cast<const char *>(r.p + r.pos), len);
    r.pos += len;
    return s;
}
inline void put_string_vector(Writer &w, const std::vector<std::string> &v) {
    put_number(w, v.size());
    for (const auto &s : v) put_string(w, s);
}
inline std::vector<std::string> get_string_vector(Reader &r) {
    const uint64_t k = get_number(r);
    if (k > r.n - r.pos) throw FormatError("string vector longer than the stream");
    std::vector<std::string> v;
    v.reserve(k);
    for (uint64_t i = 0; i < k; ++i) v.push_back(get_string(r));
    return v;
}

// ---- sdsl bit helpers ----------------------------------------------------
inline uint32_t hi_bit(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }  // x > 0
// sdsl's width for values up to v: bits::hi(v) + 1, where hi(0) = -1 gives
// width 0, which int_vector<>::width() turns into 64
inline uint8_t width_for(uint64_t v) { return v ? (uint8_t)(hi_bit(v) + 1) : (uint8_t)64; }

inline uint64_t get_bits(const std::vector<uint64_t> &w, uint64_t pos, uint32_t len) {  // len <= 64
    if (!len) return 0;
    const uint64_t i = pos >> 6, o = pos & 63;
    uint64_t v = w[i] >> o;
    if (o && o + len > 64) v |= w[i + 1] << (64 - o);
    return len == 64 ? v : v & ((1ull << len) - 1);
}
inline void set_bits(std::vector<uint64_t> &w, uint64_t pos, uint32_t len, uint64_t v) {  // len <= 64
    if (!len) return;
    const uint64_t i = pos >> 6, o = pos & 63;
    const uint64_t mask = len == 64 ? ~0ull : ((1ull << len) - 1);
    v &= mask;
    w[i] = (w[i] & ~(mask << o)) | (v << o);
    if (o && o + len > 64) {
        const uint32_t done = 64 - (uint32_t)o;
        const uint64_t m2 = mask >> done;
        w[i + 1] = (w[i + 1] & ~m2) | (v >> done);
    }
}

// ---- sdsl int_vector<> (variable width) and bit_vector -------------------
struct IntVector {
    uint64_t len = 0;  // elements
    uint8_t width = 64;
    std::vector<uint64_t> words;
    IntVector() = default;
    IntVector(uint64_t n, uint8_t w) : len(n), width(w ? w : 64), words((n * (w ? w : 64) + 63) / 64, 0) {}
    uint64_t get(uint64_t i) const { return get_bits(words, i * width, width); }
    void set(uint64_t i, uint64_t v) { set_bits(words, i * width, width, v); }
};

inline void put_int_vector(Writer &w, const IntVector &v) {
    const uint64_t bits = v.len * v.width;
    w.u64le(bits);
    w.u8(v.width);
    for (uint64_t k = 0; k < (bits + 63) / 64; ++k) w.u64le(v.words[k]);
}
inline IntVector get_int_vector(Reader &r) {
    const uint64_t bits = r.u64le();
    const uint8_t width = r.u8();
    if (width == 0 || width > 64 || bits % width) throw FormatError("int_vector: bad size/width");
    const uint64_t W = r.words_for(bits);
    IntVector v;
    v.len = bits / width;
    v.width = width;
    v.words.resize(W);
    for (uint64_t k = 0; k < W; ++k) v.words[k] = r.u64le();
    return v;
}
// bit_vector = int_vector<1>: the header has no width byte
inline void put_bit_vector(Writer &w, const std::vector<uint64_t> &words, uint64_t bits) {
    w.u64le(bits);
    for (uint64_t k = 0; k < (bits + 63) / 64; ++k) w.u64le(k < words.size() ? words[k] : 0);
}
inline std::vector<uint64_t> get_bit_vector(Reader &r, uint64_t *bits) {
    *bits = r.u64le();
    const uint64_t W = r.words_for(*bits);
    std::vector<uint64_t> words(W);
    for (uint64_t k = 0; k < W; ++k) words[k] = r.u64le();
    return words;
}

// ---- sdsl rrr_vector<63, int_vector<>, 32> -------------------------------
constexpr uint32_t kRrrBlock = 63;   // t_bs
constexpr uint32_t kRrrSample = 32;  // t_k

struct Binomial63 {
    uint64_t C[kRrrBlock + 1][kRrrBlock + 1];
    uint8_t space[kRrrBlock + 1];  // bits of a block number of class k
    Binomial63() {
        std::memset(C, 0, sizeof(C));
        for (uint32_t n = 0; n <= kRrrBlock; ++n) {
            C[n][0] = 1;
            for (uint32_t k = 1; k <= n; ++k) C[n][k] = C[n - 1][k - 1] + (k <= n - 1 ? C[n - 1][k] : 0);
        }
        for (uint32_t k = 0; k <= kRrrBlock; ++k)
            space[k] = C[kRrrBlock][k] <= 1 ? 0 : (uint8_t)(hi_bit(C[kRrrBlock][k] - 1) + 1);
    }
    // rrr_helper::bin_to_nr: rank of a 63-bit block among the blocks of its
    // class, scanning from the least significant bit
    uint64_t bin_to_nr(uint64_t bin) const {
        uint32_t k = (uint32_t)__builtin_popcountll(bin), nn = kRrrBlock;
        uint64_t nr = 0;
        while (bin) {
            if (bin & 1) {
                nr += C[nn - 1][k];
                --k;
            }
            bin >>= 1;
            --nn;
        }
        return nr;
    }
    uint64_t nr_to_bin(uint64_t nr, uint32_t k) const {
        uint64_t bin = 0;
        for (uint32_t pos = 0, nn = kRrrBlock; k && nn; ++pos, --nn) {
            const uint64_t c = C[nn - 1][k];
            if (nr >= c) {
                bin |= 1ull << pos;
                nr -= c;
                --k;
            }
        }
        return bin;
    }
};
inline const Binomial63 &binomial63() {
    static const Binomial63 b;
    return b;
}

// plain bit vector (LSB-first words, `size` bits) -> rrr_vector<63> stream
inline void put_rrr(Writer &w, const std::vector<uint64_t> &bv, uint64_t size) {
    const Binomial63 &B = binomial63();
    const uint64_t nblocks = (size + kRrrBlock) / kRrrBlock;  // + a dummy block when size % 63 == 0
    const uint64_t nsuper = (nblocks + kRrrSample - 1) / kRrrSample;
    auto block_bits = [&](uint64_t b) -> uint64_t {
        const uint64_t p = b * kRrrBlock;
        if (p >= size) return 0;
        const uint32_t len = (uint32_t)std::min<uint64_t>(kRrrBlock, size - p);
        return get_bits(bv, p, len);
    };
    IntVector bt(nblocks, 6);
    uint64_t btnr_len = 0, ones = 0;
    for (uint64_t b = 0; b < nblocks; ++b) {
        const uint32_t x = (uint32_t)__builtin_popcountll(block_bits(b));
        bt.set(b, x);
        ones += x;
        btnr_len += B.space[x];
    }
    // superblocks of 32 FULL blocks with more than 16 blocks of class > 31 are
    // stored complemented (classes 63 - x, numbers of the complemented bits)
    std::vector<uint64_t> invert((nsuper + 63) / 64, 0);
    for (uint64_t s = 0; s < nsuper; ++s) {
        const uint64_t b0 = s * kRrrSample;
        if ((b0 + kRrrSample) * kRrrBlock > size) continue;
        uint32_t gt = 0;
        for (uint64_t b = b0; b < b0 + kRrrSample; ++b) gt += bt.get(b) > kRrrBlock / 2;
        if (gt > kRrrSample / 2) {
            invert[s >> 6] |= 1ull << (s & 63);
            for (uint64_t b = b0; b < b0 + kRrrSample; ++b) bt.set(b, kRrrBlock - bt.get(b));
        }
    }
    std::vector<uint64_t> btnr((std::max<uint64_t>(btnr_len, 64) + 63) / 64, 0);
    IntVector btnrp(nsuper, width_for(btnr_len));
    IntVector rank(nsuper + ((size % ((uint64_t)kRrrSample * kRrrBlock)) > 0), width_for(ones));
    uint64_t pos = 0, sum = 0;
    for (uint64_t b = 0; b < nblocks; ++b) {
        const uint64_t s = b / kRrrSample;
        const bool inv = (invert[s >> 6] >> (s & 63)) & 1;
        if (b % kRrrSample == 0) {
            btnrp.set(s, pos);
            rank.set(s, sum);
        }
        const uint32_t x = (uint32_t)bt.get(b);
        uint64_t bin = block_bits(b);
        if (inv) bin = ~bin & ((1ull << kRrrBlock) - 1);
        sum += inv ? kRrrBlock - x : x;
        if (B.space[x]) set_bits(btnr, pos, B.space[x], B.bin_to_nr(bin));
        pos += B.space[x];
    }
    if (rank.len > nsuper) rank.set(rank.len - 1, sum);
    w.u64le(size);
    put_int_vector(w, bt);
    put_bit_vector(w, btnr, std::max<uint64_t>(btnr_len, 64));
    put_int_vector(w, btnrp);
    put_int_vector(w, rank);
    put_bit_vector(w, invert, nsuper);
}

// rrr_vector<63> stream -> plain bit vector (LSB-first words)
inline std::vector<uint64_t> get_rrr(Reader &r, uint64_t *size_out) {
    const Binomial63 &B = binomial63();
    const uint64_t size = r.u64le();
    const IntVector bt = get_int_vector(r);
    uint64_t btnr_bits = 0, inv_bits = 0;
    const std::vector<uint64_t> btnr = get_bit_vector(r, &btnr_bits);
    (void)get_int_vector(r);  // btnrp: samples, recomputed while decoding
    (void)get_int_vector(r);  // rank samples
    const std::vector<uint64_t> invert = get_bit_vector(r, &inv_bits);
    // the size is untrusted: the block classes (read from the stream) bound it
    if (size / kRrrBlock > bt.len) throw FormatError("rrr_vector: size larger than its blocks");
    const uint64_t nblocks = (size + kRrrBlock) / kRrrBlock;
    if (bt.len < nblocks || (size > 0 && bt.len > nblocks + 1)) throw FormatError("rrr_vector: block count");
    std::vector<uint64_t> out((size + 63) / 64 + 1, 0);
    uint64_t pos = 0;
    for (uint64_t b = 0; b < nblocks; ++b) {
        const uint64_t s = b / kRrrSample;
        const bool inv = s < inv_bits && ((invert[s >> 6] >> (s & 63)) & 1);
        const uint32_t x = (uint32_t)bt.get(b);
        if (x > kRrrBlock) throw FormatError("rrr_vector: block class > 63");
        const uint32_t sp = B.space[x];
        if (pos + sp > btnr_bits) throw FormatError("rrr_vector: block numbers past the end");
        const uint64_t nr = get_bits(btnr, pos, sp);
        if (nr >= B.C[kRrrBlock][x]) throw FormatError("rrr_vector: block number out of range");
        pos += sp;
        uint64_t bin = B.nr_to_bin(nr, x);
        if (inv) bin = ~bin & ((1ull << kRrrBlock) - 1);
        const uint64_t p = b * kRrrBlock;
        if (p >= size) break;
        const uint32_t len = (uint32_t)std::min<uint64_t>(kRrrBlock, size - p);
        set_bits(out, p, len, bin);
    }
    out.resize((size + 63) / 64);
    *size_out = size;
    return out;
}

}  // namespace fmt
}  // namespace mbrwt

namespace mbrwt {
namespace fmt {

// ---- sdsl int_vector<64> (fixed width: the header has no width byte) -----
inline void put_int_vector64(Writer &w, const std::vector<uint64_t> &v) {
    w.u64le((uint64_t)v.size() * 64);
    for (uint64_t x : v) w.u64le(x);
}
inline std::vector<uint64_t> get_int_vector64(Reader &r) {
    const uint64_t bits = r.u64le();
    if (bits % 64) throw FormatError("int_vector<64>: size not a multiple of 64 bits");
    const uint64_t W = r.words_for(bits);
    std::vector<uint64_t> v(W);
    for (uint64_t k = 0; k < W; ++k) v[k] = r.u64le();
    return v;
}

// ---- sdsl wt_int<rrr_vector<63>> ------------------------------------------
// (BinRelWT_sdsl::wt_, bin_rel_wt_sdsl.hpp:40; construct_im at
// bin_rel_wt_sdsl.cpp:39.)  sdsl-lite's published layout: {u64 size, u64
// sigma (the effective alphabet: distinct symbols), rrr_vector<63> tree of
// size * max_level bits, the rrr rank/select supports (no bytes), u32
// max_level, int_vector<64> zero_cnt (zeros per level), int_vector<64>
// rank_level (ones before each level)}.  Level l of the tree holds bit
// max_level - 1 - l of every symbol, the symbols stably ordered by their top l
// bits (the wavelet tree's nodes side by side); max_level = bits of
// max(1, largest symbol).  An empty sequence keeps the defaults of a
// default-constructed wt_int (its constructor returns before max_level is
// computed): max_level 0, an empty tree and empty level vectors.  PARITY
// UNPINNED like the rest of this file.
inline void put_wt_int(Writer &w, const std::vector<uint64_t> &seq) {
    const uint64_t n = seq.size();
    uint64_t mx = 1;
    for (uint64_t x : seq) mx = std::max(mx, x);
    const uint32_t levels = n ? hi_bit(mx) + 1 : 0;
    std::vector<uint64_t> sorted(seq);
    std::sort(sorted.begin(), sorted.end());
    const uint64_t sigma = n ? (uint64_t)(std::unique(sorted.begin(), sorted.end()) - sorted.begin()) : 0;
    std::vector<uint64_t> tree((n * levels + 63) / 64 + 1, 0), zero_cnt(levels, 0), rank_level(levels, 0);
    std::vector<uint64_t> cur(seq), nxt(n);
    uint64_t ones = 0;
    for (uint32_t l = 0; l < levels; ++l) {
        const uint32_t bit = levels - 1 - l;
        rank_level[l] = ones;
        // nodes: runs of equal top-l prefixes in `cur`; each is split stably
        uint64_t i = 0;
        while (i < n) {
            const uint64_t pre = (l ? cur[i] >> (bit + 1) : 0);
            uint64_t j = i;
            while (j < n && (l ? cur[j] >> (bit + 1) : 0) == pre) ++j;
            uint64_t z = i;
            for (uint64_t k = i; k < j; ++k) {
                const uint64_t b = (cur[k] >> bit) & 1;
                if (b) {
                    tree[(l * n + k) >> 6] |= 1ull << ((l * n + k) & 63);
                    ++ones;
                } else {
                    nxt[z++] = cur[k];
                }
            }
            zero_cnt[l] += z - i;
            for (uint64_t k = i; k < j; ++k)
                if ((cur[k] >> bit) & 1) nxt[z++] = cur[k];
            i = j;
        }
        cur.swap(nxt);
    }
    w.u64le(n);
    w.u64le(sigma);
    tree.resize((n * levels + 63) / 64);
    put_rrr(w, tree, n * levels);
    const uint32_t ml = levels;
    w.bytes(&ml, 4);
    put_int_vector64(w, zero_cnt);
    put_int_vector64(w, rank_level);
}

inline std::vector<uint64_t> get_wt_int(Reader &r) {
    const uint64_t n = r.u64le();
    (void)r.u64le();  // sigma
    uint64_t tbits = 0;
    const std::vector<uint64_t> tree = get_rrr(r, &tbits);
    uint32_t levels = 0;
    r.bytes(&levels, 4);
    const std::vector<uint64_t> zero_cnt = get_int_vector64(r), rank_level = get_int_vector64(r);
    if (levels == 0 && n == 0 && tbits == 0 && zero_cnt.empty() && rank_level.empty()) return {};  // empty wt_int
    if (levels == 0 || levels > 64) throw FormatError("wt_int: bad max_level");
    if (tbits % levels || tbits / levels != n) throw FormatError("wt_int: tree size != size * max_level");
    if (zero_cnt.size() != levels || rank_level.size() != levels) throw FormatError("wt_int: level vectors");
    // decode: order[k] = the sequence position of the k-th symbol of the
    // current level; every level's stable split refines the order
    std::vector<uint64_t> val(n, 0), order(n), nxt(n), pre(n, 0);
    for (uint64_t k = 0; k < n; ++k) order[k] = k;
    uint64_t ones = 0;
    for (uint32_t l = 0; l < levels; ++l) {
        if (rank_level[l] != ones) throw FormatError("wt_int: rank_level mismatch");
        uint64_t i = 0, zeros = 0;
        while (i < n) {
            uint64_t j = i;
            while (j < n && pre[order[j]] == pre[order[i]]) ++j;
            uint64_t z = i;
            for (uint64_t k = i; k < j; ++k) {
                const uint64_t p = l * n + k;
                const uint64_t b = (tree[p >> 6] >> (p & 63)) & 1;
                val[order[k]] = (val[order[k]] << 1) | b;
                if (!b) nxt[z++] = order[k];
                ones += b;
            }
            zeros += z - i;
            for (uint64_t k = i; k < j; ++k)
                if (val[order[k]] & 1) nxt[z++] = order[k];
            i = j;
        }
        if (zero_cnt[l] != zeros) throw FormatError("wt_int: zero_cnt mismatch");
        order.swap(nxt);
        for (uint64_t k = 0; k < n; ++k) pre[k] = val[k];
    }
    return val;
}

}  // namespace fmt
}  // namespace mbrwt
