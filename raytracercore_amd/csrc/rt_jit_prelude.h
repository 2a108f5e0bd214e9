// rt_jit_prelude.h -- first header of the scene-specialised kernels compiled at run time by
// hiprtc (rt_jit.cpp): hiprtc declares the fixed-width integer types in its own namespace.
#pragma once
#ifdef __HIPCC_RTC__
typedef __hip_internal::int8_t int8_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::int16_t int16_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
#endif
