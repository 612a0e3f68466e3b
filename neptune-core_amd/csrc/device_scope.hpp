// Every entry point that works on a context's device makes it current for the call and puts the
// caller's current device back on return: a host with its own HIP user on the same thread (torch,
// another library) never finds a different device current after calling into neptune_hip.
#pragma once
#include <hip/hip_runtime.h>

struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};
