// Named host-side trace ranges (epochs, halo exchanges, polls).  The engine
// is plain C++; the HIP backend installs roctx hooks (rocprofiler-sdk-roctx)
// so the ranges show up in `rocprofv3 --marker-trace`.  Without hooks the
// ranges cost two predictable branches.
#pragma once

namespace gol {
namespace trace {

using PushFn = void (*)(const char*);
using PopFn = void (*)();

void set_hooks(PushFn push, PopFn pop);
void push(const char* name);
void pop();

struct Range {
  explicit Range(const char* name) { push(name); }
  ~Range() { pop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

}  // namespace trace
}  // namespace gol
