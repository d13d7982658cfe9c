// annotate_static.hpp -- C++ host mirror of the reference's static
// annotator over any BinaryMatrix, used with BRWTDevice for the device path.
//
// Restated interfaces (ratschlab/genome_graph_annotation):
//   LabelEncoder<Label>                  common/annotate.hpp:110-140, annotate.cpp:12-31
//   MultiLabelEncoded::get_top_labels    common/annotate.cpp:57-83
//   StaticBinRelAnnotator<Matrix>        annotation/annotate_static.{hpp,cpp}
//     has_label :26-33, has_labels :35-55, get_labels(i) :57-67,
//     get_labels(indices, ratio) :71-94, count_labels :149-162
// count_labels (the `classify` hot loop, annotate_static.cpp:155-159) goes
// through the matrix's batched get_rows(), i.e. one device launch for the
// whole index list instead of one get_row per index.
#pragma once

#include <algorithm>
#include <cassert>
#include <cmath>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "brwt_device.hpp"

namespace mbrwt_host {

template <typename Label = std::string>
class LabelEncoder {
  public:
    // annotate.cpp:23-31
    size_t insert_and_encode(const Label &label) {
        auto it = encode_label_.find(label);
        if (it != encode_label_.end()) return it->second;
        encode_label_[label] = decode_label_.size();
        decode_label_.push_back(label);
        return decode_label_.size() - 1;
    }
    // annotate.cpp:12-20: throws if the label does not exist
    size_t encode(const Label &label) const {
        auto it = encode_label_.find(label);
        if (it == encode_label_.end()) throw std::runtime_error("ERROR: No such label");
        return it->second;
    }
    // annotate.hpp:128: throws on a bad code
    const Label &decode(size_t code) const { return decode_label_.at(code); }
    size_t size() const { return decode_label_.size(); }
    void clear() {
        encode_label_.clear();
        decode_label_.clear();
    }

  private:
    std::unordered_map<Label, uint64_t> encode_label_;
    std::vector<Label> decode_label_;
};

template <class Matrix, typename Label = std::string>
class StaticBinRelAnnotator {
  public:
    typedef uint64_t Index;
    typedef std::vector<Label> VLabels;

    StaticBinRelAnnotator(std::shared_ptr<const Matrix> matrix, const LabelEncoder<Label> &label_encoder)
        : matrix_(std::move(matrix)), label_encoder_(label_encoder) {
        if (!matrix_) throw std::invalid_argument("null matrix");
    }

    // annotate_static.cpp:26-33
    bool has_label(Index i, const Label &label) const {
        try {
            return matrix_->get(i, label_encoder_.encode(label));
        } catch (const std::out_of_range &) {
            throw;
        } catch (...) {
            return false;
        }
    }

    // annotate_static.cpp:35-55
    bool has_labels(Index i, const VLabels &labels) const {
        std::set<size_t> querying_codes;
        try {
            for (const auto &label : labels) querying_codes.insert(label_encoder_.encode(label));
        } catch (...) {
            return false;
        }
        std::set<size_t> encoded_labels;
        for (auto col : matrix_->get_row(i)) encoded_labels.insert(col);
        return std::includes(encoded_labels.begin(), encoded_labels.end(), querying_codes.begin(),
                             querying_codes.end());
    }

    // annotate_static.cpp:57-67
    VLabels get_labels(Index i) const {
        VLabels labels;
        for (auto col : matrix_->get_row(i)) labels.push_back(label_encoder_.decode(col));
        return labels;
    }

    // annotate_static.cpp:71-94: labels present in at least
    // ceil(|indices| * presence_ratio) rows (any row if the ratio is 0)
    VLabels get_labels(const std::vector<Index> &indices, double presence_ratio) const {
        assert(presence_ratio >= 0 && presence_ratio <= 1);
        const size_t min_labels_discovered =
            presence_ratio == 0 ? 1 : (size_t)std::ceil(indices.size() * presence_ratio);
        auto counts = count_labels(indices);
        VLabels filtered;
        for (size_t i = 0; i < counts.size(); ++i)
            if (counts[i] && counts[i] >= min_labels_discovered) filtered.push_back(label_encoder_.decode(i));
        return filtered;
    }

    // get_labels(indices, presence_ratio) for a batch of reads (the classify
    // loop over reads, annotated_dbg.cpp:88-110): one device call for all
    // reads when the matrix offers it (BRWTDevice, BinRelWTDevice), else one
    // get_labels per read
    std::vector<VLabels> get_labels_batch(const std::vector<std::vector<Index>> &reads,
                                          double presence_ratio) const {
        assert(presence_ratio >= 0 && presence_ratio <= 1);
        std::vector<Index> rows;
        std::vector<uint64_t> read_off{0}, lab_off;
        for (const auto &read : reads) {
            rows.insert(rows.end(), read.begin(), read.end());
            read_off.push_back(rows.size());
        }
        std::vector<uint32_t> codes;
        std::vector<VLabels> out(reads.size());
        if (!matrix_->labels_batch_csr(rows, read_off, presence_ratio, &lab_off, &codes)) {
            for (size_t r = 0; r < reads.size(); ++r) out[r] = get_labels(reads[r], presence_ratio);
            return out;
        }
        for (size_t r = 0; r < reads.size(); ++r)
            for (uint64_t i = lab_off[r]; i < lab_off[r + 1]; ++i) out[r].push_back(label_encoder_.decode(codes[i]));
        return out;
    }

    // annotate.cpp:57-83 (std::sort: ties in unspecified order, as in the reference)
    std::vector<std::pair<Label, size_t>> get_top_labels(const std::vector<Index> &indices,
                                                         size_t num_top = static_cast<size_t>(-1)) const {
        auto counter = count_labels(indices);
        std::vector<std::pair<size_t, size_t>> counts;
        for (size_t j = 0; j < counter.size(); ++j)
            if (counter[j]) counts.emplace_back(j, counter[j]);
        std::sort(counts.begin(), counts.end(),
                  [](const auto &a, const auto &b) { return a.second > b.second; });
        counts.resize(std::min(counts.size(), num_top));
        std::vector<std::pair<Label, size_t>> top;
        for (const auto &p : counts) top.emplace_back(label_encoder_.decode(p.first), p.second);
        return top;
    }

    // get_top_labels for a batch of reads (classify --count-labels,
    // main.cpp:177): one device call when the matrix offers it, else one
    // get_top_labels per read
    std::vector<std::vector<std::pair<Label, size_t>>> get_top_labels_batch(
        const std::vector<std::vector<Index>> &reads, size_t num_top = static_cast<size_t>(-1)) const {
        std::vector<Index> rows;
        std::vector<uint64_t> read_off{0}, lab_off, counts;
        for (const auto &read : reads) {
            rows.insert(rows.end(), read.begin(), read.end());
            read_off.push_back(rows.size());
        }
        std::vector<uint32_t> codes;
        std::vector<std::vector<std::pair<Label, size_t>>> out(reads.size());
        if (!matrix_->top_labels_batch_csr(rows, read_off, num_top, &lab_off, &codes, &counts)) {
            for (size_t r = 0; r < reads.size(); ++r) out[r] = get_top_labels(reads[r], num_top);
            return out;
        }
        for (size_t r = 0; r < reads.size(); ++r)
            for (uint64_t i = lab_off[r]; i < lab_off[r + 1]; ++i)
                out[r].emplace_back(label_encoder_.decode(codes[i]), counts[i]);
        return out;
    }

    uint64_t num_objects() const { return matrix_->num_rows(); }
    size_t num_labels() const { return label_encoder_.size(); }
    uint64_t num_relations() const { return matrix_->num_relations(); }
    const Matrix &data() const { return *matrix_; }

    // annotate_static.cpp:149-162, batched
    std::vector<uint64_t> count_labels(const std::vector<Index> &indices) const {
        std::vector<uint64_t> counter(num_labels(), 0);
        if (indices.empty()) return counter;
        for (const auto &row : matrix_->get_rows(indices))
            for (auto col : row) counter[col]++;
        return counter;
    }

  private:
    std::shared_ptr<const Matrix> matrix_;
    LabelEncoder<Label> label_encoder_;
};

}  // namespace mbrwt_host
