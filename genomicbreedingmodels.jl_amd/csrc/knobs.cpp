// Tuning and test knobs (GBM_* environment variables) without getenv on the fit path.
//
// The library is called concurrently from Julia's Threads.@threads (reference
// src/cross_validation.jl:159); a getenv racing a setenv in another thread is undefined behaviour.
// So the environment is read ONCE, at the first knob lookup (every GBM_* entry of environ is copied
// into a table), and afterwards the table changes only through gbm_debug_set (tests, A/B timing
// runs), under a reader/writer lock. Values are interned (never freed), so the pointer knob()
// returns stays valid for the life of the process even if a later gbm_debug_set replaces it.
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>

#include "gbm_internal.h"

extern char** environ;

namespace gbm {
namespace {

struct KnobTable {
  std::shared_mutex mu;
  std::map<std::string, const char*> vals;  // interned values; absent = unset
  std::once_flag once;
};

KnobTable& table() {
  static KnobTable* t = new KnobTable();  // never destroyed: knobs may be read during static teardown
  return *t;
}

const char* intern(const char* v) {
  const size_t len = strlen(v);
  char* p = new char[len + 1];
  memcpy(p, v, len + 1);
  return p;
}

void snapshot(KnobTable& t) {
  for (char** e = environ; e && *e; e++) {
    if (strncmp(*e, "GBM_", 4) != 0) continue;
    const char* eq = strchr(*e, '=');
    if (!eq) continue;
    t.vals[std::string(*e, eq - *e)] = intern(eq + 1);
  }
}

}  // namespace

const char* knob(const char* name) {
  KnobTable& t = table();
  std::call_once(t.once, [&] {
    std::unique_lock<std::shared_mutex> lk(t.mu);
    snapshot(t);
  });
  std::shared_lock<std::shared_mutex> lk(t.mu);
  auto it = t.vals.find(name);
  return it == t.vals.end() ? nullptr : it->second;
}

int64_t knob_i64(const char* name, int64_t def) {
  const char* e = knob(name);
  return e && *e ? (int64_t)atoll(e) : def;
}

}  // namespace gbm

extern "C" int gbm_debug_set(const char* name, const char* value) {
  if (!name || strncmp(name, "GBM_", 4) != 0) return gbm::fail(GBM_E_ARG, "gbm_debug_set: the knob name must start with GBM_");
  gbm::KnobTable& t = gbm::table();
  (void)gbm::knob(name);  // the environment snapshot first, so a later first lookup cannot overwrite this set
  std::unique_lock<std::shared_mutex> lk(t.mu);
  if (value)
    t.vals[name] = gbm::intern(value);
  else
    t.vals.erase(name);
  return GBM_OK;
}
