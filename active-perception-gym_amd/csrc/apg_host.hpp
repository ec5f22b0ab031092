// apg_host.hpp — host-side helpers shared by the translation units of libapgym_hip.so.
#pragma once
#include <hip/hip_runtime.h>

namespace apg {
// Record `msg` as apg_last_error() and return `code`.
int fail(int code, const char *msg);
// APG_OK, or APG_E_LAUNCH with the HIP error of the last launch recorded under `what`.
int check_launch(const char *what);
}  // namespace apg
