// Workspace carving shared by the plans: a dry pass sizes the workspace, a bound pass hands out aligned pointers.
#pragma once
#include "common.h"

namespace vad {

struct Ws {
  char* base = nullptr;
  int64_t off = 0;
  bool dry = true;
  template <class T>
  T* take(int64_t n) {
    off = (off + 255) / 256 * 256;
    T* p = dry ? nullptr : reinterpret_cast<T*>(base + off);
    off += n * (int64_t)sizeof(T);
    return p;
  }
};

}  // namespace vad
