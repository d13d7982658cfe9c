// device_access.hpp -- typed global/LDS accesses for the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace mbrwt {

// Explicit address spaces: image addresses are rebuilt from integers and
// would otherwise compile to flat_* loads, which CDNA4 retires out of order
// (every wait becomes vmcnt(0) & lgkmcnt(0)).  Every hot access below is a
// global_* (address space 1) or ds_* (address space 3) instruction.
#define AS_GLOBAL __attribute__((address_space(1)))
#define AS_LDS __attribute__((address_space(3)))
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// (the host pass of the same source only needs the declarations to parse)
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
__device__ __forceinline__ T gld(const T *p) { return *(const AS_GLOBAL T *)(uintptr_t)p; }
template <class T>
__device__ __forceinline__ T gld_at(uint64_t addr) { return *(const AS_GLOBAL T *)addr; }
template <class T>
__device__ __forceinline__ void gst(T *p, T v) { *(AS_GLOBAL T *)(uintptr_t)p = v; }
template <class T, bool NT>
__device__ __forceinline__ T gld_at_nt(uint64_t addr) {
    if constexpr (!NT) {
        return *(const AS_GLOBAL T *)addr;
    } else if constexpr (sizeof(T) == 16) {
        const u32x4_t v = __builtin_nontemporal_load((const AS_GLOBAL u32x4_t *)addr);
        return T{v.x, v.y, v.z, v.w};
    } else if constexpr (sizeof(T) == 8 && !std::is_integral<T>::value) {
        const u32x2_t v = __builtin_nontemporal_load((const AS_GLOBAL u32x2_t *)addr);
        return T{v.x, v.y};
    } else {
        return __builtin_nontemporal_load((const AS_GLOBAL T *)addr);
    }
}
#else
template <class T, bool NT>
__device__ T gld_at_nt(uint64_t addr) { return *(const T *)addr; }
template <class T>
__device__ T gld(const T *p) { return *p; }
template <class T>
__device__ T gld_at(uint64_t addr) { return *(const T *)addr; }
template <class T>
__device__ void gst(T *p, T v) { *p = v; }
#endif

}  // namespace mbrwt
