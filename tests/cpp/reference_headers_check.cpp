// Compiled (syntax and template instantiation only) against the REFERENCE's
// own common/annotate.hpp by tests/test_reference_headers.py: with
// MBRWT_WITH_REFERENCE_ANNOTATE the mirror's static annotator derives from
// the reference's annotate::MultiLabelEncoded and implements every pure
// virtual of it, so the reference's AnnotatedDBG can hold it unchanged.
#include <string>
#include <type_traits>

#include "../../genome_graph_annotation_amd/csrc/annotate_static.hpp"

using DeviceAnnotator = mbrwt_host::StaticBinRelAnnotator<mbrwt_host::BRWTDevice, std::string>;

static_assert(std::is_base_of<annotate::MultiLabelEncoded<uint64_t, std::string>, DeviceAnnotator>::value,
              "derives from the reference's MultiLabelEncoded");
static_assert(std::is_base_of<annotate::MultiLabelAnnotation<uint64_t, std::string>, DeviceAnnotator>::value,
              "is a reference MultiLabelAnnotation");
static_assert(!std::is_abstract<DeviceAnnotator>::value, "implements every pure virtual of the reference interface");

int main() {
    DeviceAnnotator a;
    annotate::MultiLabelAnnotation<uint64_t, std::string> *as_reference = &a;
    (void)as_reference->num_labels();
    return 0;
}
