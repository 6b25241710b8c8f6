// rtg_device.cuh -- device-side load/store helpers and the launch-grid helper shared by the kernel TUs.
#pragma once
#include "rtg_kernels.cuh"

namespace rtg {

// ----------------------------------------------------------------------------
// loads / stores
// ----------------------------------------------------------------------------
RTG_DEV V ld3(const float *__restrict__ p) { return V{p[0], p[1], p[2]}; }
RTG_DEV Q ld4(const float *__restrict__ p)
{
    const float4 v = *reinterpret_cast<const float4 *>(p);
    return Q{v.x, v.y, v.z, v.w};
}
RTG_DEV void st4(float *__restrict__ p, Q q) { *reinterpret_cast<float4 *>(p) = make_float4(q.x, q.y, q.z, q.w); }
RTG_DEV void st3(float *__restrict__ p, V v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

// Launch-uniform tables (topology, schedule) read through the constant address
// space: the compiler cannot prove them unclobbered in a kernel that stores to
// global memory, so a plain load would be a vector load, and its s_waitcnt
// vmcnt would also drain every prefetch in flight.  These become s_load (lgkmcnt).
template <typename T>
RTG_DEV T ld_const(const T *p)
{
    return *(const __attribute__((address_space(4))) T *)p;
}
RTG_DEV V ld_const(const V *p) { return V{ld_const(&p->x), ld_const(&p->y), ld_const(&p->z)}; }
RTG_DEV Q ld_const(const Q *p) { return Q{ld_const(&p->x), ld_const(&p->y), ld_const(&p->z), ld_const(&p->w)}; }

static inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

}  // namespace rtg
