// Experiment knobs of the native library (see utils/knobs.py): an NNMPI_* environment variable
// that selects a kernel variant or policy is read only when NNMPI_EXPERIMENTS=1, so a stray
// variable on a benchmark box cannot change what is timed.  The set_* entry points of the
// bindings (kernel-selection knobs for A/B scripts) are gated the same way.
#pragma once
#include <cstdlib>

// 1 in the experiments library only (_build.py, NNMPI_BUILD_EXPERIMENTS=1): the diagnostic
// stamped kernel twins, the in-launch split-K fixup and the half-width weight-gradient tile --
// measured, kept for re-measurement, never on the training path -- are compiled in only there.
#ifndef NNMPI_EXPERIMENTS_BUILD
#define NNMPI_EXPERIMENTS_BUILD 0
#endif

namespace nnmpi {

inline bool experiments_on() {
  static const bool on = [] {
    const char* e = std::getenv("NNMPI_EXPERIMENTS");
    return e && e[0] == '1' && e[1] == '\0';
  }();
  return on;
}

// getenv for an experiment knob: null unless experiments are on
inline const char* knob_env(const char* name) { return experiments_on() ? std::getenv(name) : nullptr; }

}  // namespace nnmpi
