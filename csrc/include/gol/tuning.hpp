// Runtime tuning: every knob that is not part of the simulation itself
// (EngineConfig) - kernel and schedule choice, launch planning, diagnostics,
// fault injection, the CPU backend's emulation of device features.
//
// One table (tuning_keys(), tuning.cpp) names each knob once: its key
// (`--tune key=value` on bin/gol, bench.py and gol_amd.cli; LifeConfig.tune),
// the GOL_* environment variable that may override its default, the default,
// its class and what it does.  Effective value, lowest to highest precedence:
// the table's default, the environment (read by Tuning::from_env and nowhere
// else in the framework), explicit settings (Tuning::set).  Backends read
// their knobs from the Tuning they are constructed with, the engine from
// EngineConfig::tune, the transports and tools from Tuning::from_env() at
// construction: a knob never changes under a live object.
//
// Classes:
//   tune          performance knobs of the default build (the measured-
//                 slower variants and their probes were removed in round 6,
//                 HISTORY.md);
//   diag          traces, logs and consistency checks;
//   fault         fault injection (tests);
//   emul          the CPU backend emulating a device feature (tests).
//
// The reference has no runtime tuning: its block size, grid size and the
// OpenMP schedule are compile-time constants (src/game_cuda.cu:12-14,
// src/game_openmp.c:95).
#pragma once

#include <map>
#include <string>
#include <utility>
#include <vector>

namespace gol {

struct TuningKey {
  const char* key;
  const char* env;
  const char* dflt;
  char type;        // 'i' integer, 'f' number, 's' string
  const char* cls;  // tune | diag | fault | emul
  const char* doc;
};
const std::vector<TuningKey>& tuning_keys();

class Tuning {
 public:
  Tuning();  // every key at its default
  // Defaults overlaid by the GOL_* variables that are set (non-empty).
  static Tuning from_env();

  // key=value (unknown keys, and values that do not parse as the key's type,
  // fail with the key and its GOL_* variable named).  from_env() validates
  // every GOL_* variable that is set, so a malformed one fails whichever
  // component reads the tuning first.
  Tuning& set(const std::string& key, const std::string& value);
  Tuning& set(const std::string& kv);

  int i(const std::string& key) const;
  double f(const std::string& key) const;
  const std::string& s(const std::string& key) const;
  bool on(const std::string& key) const { return i(key) != 0; }
  bool is_default(const std::string& key) const;
  const std::string& source(const std::string& key) const;  // default | env | set

  const std::map<std::string, std::string>& values() const { return v_; }
  // Keys off their default: key -> value.
  std::map<std::string, std::string> changed() const;
  // "key=value[source] ..." of the changed keys ("defaults" when none).
  std::string summary() const;

 private:
  std::map<std::string, std::string> v_, src_;
};

}  // namespace gol
