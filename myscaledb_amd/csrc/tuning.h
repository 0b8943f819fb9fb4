// tuning.h -- A/B switches for measurement builds only.
//
// The release library (libmqvs.so) never reads the environment: every switch
// below returns its default there, so no variable in a server's environment
// can change a kernel or select a diagnostic build.  The measurement build
// (`make dbg` -> libmqvs_dbg.so, compiled with -DMQVS_DEBUG_TUNING) reads
// them with getenv; tools load it only through an explicit
// myscaledb_amd._lib.use_measurement_build() call (their --dbg option).
#pragma once

#include <cstdlib>

namespace mqvs {

#ifdef MQVS_DEBUG_TUNING
constexpr bool kDebugTuning = true;
inline const char *tune_env(const char *name) { return std::getenv(name); }
#else
constexpr bool kDebugTuning = false;
inline const char *tune_env(const char *) { return nullptr; }
#endif

// integer switch: the variable's value in a measurement build, dflt otherwise
inline int tune_int(const char *name, int dflt) {
    const char *e = tune_env(name);
    return (e && *e) ? std::atoi(e) : dflt;
}

}  // namespace mqvs
