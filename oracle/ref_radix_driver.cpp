// ref_radix_driver.cpp — TEST INFRASTRUCTURE (oracle/_ref).
//
// Exposes the reference's own CPU radix sort + grouping (include/gpu_depthmap_fusion/
// radix_grouper.h:5-67 and radix_sort.h:107-289, compiled unmodified from /root/reference by
// oracle/Makefile) through a C entry point, so the oracle's stable-sort restatement and the GPU
// voxelize can be pinned against the reference's actual code.  The only thing supplied here is
// the TUintVec4 template argument (the reference instantiates it with cv::Vec<uint,4>,
// gpu_depthmap_fusion.h:506); it is a template parameter of RadixSorter, not a stand-in header.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "radix_grouper.h"

struct RefUVec4 {
    uint32_t v[4];
    RefUVec4() : v{0, 0, 0, 0} {}
    RefUVec4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) : v{a, b, c, d} {}
    uint32_t& operator[](int i) { return v[i]; }
    const uint32_t& operator[](int i) const { return v[i]; }
    RefUVec4 operator+(const RefUVec4& o) const {
        return RefUVec4(v[0] + o.v[0], v[1] + o.v[1], v[2] + o.v[2], v[3] + o.v[3]);
    }
    RefUVec4& operator+=(const RefUVec4& o) {
        for (int i = 0; i < 4; ++i) v[i] += o.v[i];
        return *this;
    }
};

extern "C" int ref_radix_group(const uint32_t* keys, uint32_t n, int group_size,
                               uint32_t* sorted_idx, uint32_t* sorted_keys,
                               uint32_t* group_starts, uint32_t* group_sizes,
                               uint32_t* group_values, uint32_t* num_groups) {
    RadixGrouper<uint32_t, RefUVec4> grouper(group_size);
    grouper.group(keys, (int)n);
    for (uint32_t i = 0; i < n; ++i) {
        sorted_idx[i] = grouper.sorter.sortedIndices[i];
        sorted_keys[i] = grouper.sorter.sortedValues[i];
    }
    uint32_t g = (uint32_t)grouper.groupStarts.size();
    for (uint32_t i = 0; i < g; ++i) {
        group_starts[i] = grouper.groupStarts[i];
        group_sizes[i] = grouper.groupSizes[i];
        group_values[i] = grouper.groupValues[i];
    }
    *num_groups = g;
    return 0;
}
