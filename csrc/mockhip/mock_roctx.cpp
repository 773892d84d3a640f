// Stand-in for librocprofiler-sdk-roctx in the CPU suite: every marker and
// range the shim emits is appended as one line to $MOCK_ROCTX_OUT, so the
// tests can check what a rocprofv3 --marker-trace run would show.
#include <stdio.h>
#include <stdlib.h>

namespace {
void emit(const char* kind, const char* msg) {
  const char* path = getenv("MOCK_ROCTX_OUT");
  if (!path) return;
  FILE* f = fopen(path, "a");
  if (!f) return;
  fprintf(f, "%s %s\n", kind, msg ? msg : "");
  fclose(f);
}
}  // namespace

extern "C" __attribute__((visibility("default"))) void roctxMarkA(const char* m) { emit("mark", m); }
extern "C" __attribute__((visibility("default"))) int roctxRangePushA(const char* m) {
  emit("push", m);
  return 0;
}
extern "C" __attribute__((visibility("default"))) int roctxRangePop() {
  emit("pop", nullptr);
  return 0;
}
