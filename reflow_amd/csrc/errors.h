// errors.h -- internal: rf_last_error() state and the argument-check macro,
// shared by every translation unit of the library, the HIP-free host units
// (wire.cpp, partition_split.cpp) included.  Not part of the public ABI.
#pragma once
#include "reflow_hip.h"

namespace rf {
// Sets the thread-local rf_last_error() message; returns code.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}  // namespace rf

#define ARG(cond, msg)                                       \
    do {                                                     \
        if (!(cond)) return rf::fail(RF_EINVAL, "%s", msg); \
    } while (0)
