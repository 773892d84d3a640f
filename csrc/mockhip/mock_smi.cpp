// Mock libamd_smi / librocm_smi64 for the CPU test-suite (never shipped):
// the memory queries the shim virtualises plus the PCI-location queries it
// maps a device with.  One device, handle (void*)1 / index 0:
//   MOCKSMI_BDF        "dddd:bb:dd.f" (default 0000:75:00.0)
//   MOCKSMI_TOTAL_MIB  physical VRAM (default 294912, an MI355X)
//   MOCKSMI_USED_MIB   physical VRAM in use (default 5000)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

namespace {
uint64_t env_mib(const char* k, uint64_t d) {
  const char* v = getenv(k);
  return (v ? strtoull(v, nullptr, 10) : d) << 20;
}
uint64_t bdf_fields(unsigned* dom, unsigned* bus, unsigned* dev, unsigned* fn) {
  const char* v = getenv("MOCKSMI_BDF");
  *dom = 0, *bus = 0x75, *dev = 0, *fn = 0;
  if (v) sscanf(v, "%x:%x:%x.%x", dom, bus, dev, fn);
  return 0;
}
}  // namespace

extern "C" {
#define EXPORT __attribute__((visibility("default")))
EXPORT int amdsmi_get_gpu_device_bdf(void* h, uint64_t* bdf) {
  if (h != (void*)1 || !bdf) return 2;
  unsigned dom, bus, dev, fn;
  bdf_fields(&dom, &bus, &dev, &fn);
  *bdf = (uint64_t)fn | ((uint64_t)dev << 3) | ((uint64_t)bus << 8) | ((uint64_t)dom << 16);
  return 0;
}
EXPORT int amdsmi_get_gpu_memory_total(void* h, int type, uint64_t* total) {
  if (h != (void*)1 || !total) return 2;
  *total = type == 2 ? (512ull << 30) : env_mib("MOCKSMI_TOTAL_MIB", 294912);
  return 0;
}
EXPORT int amdsmi_get_gpu_memory_usage(void* h, int type, uint64_t* used) {
  if (h != (void*)1 || !used) return 2;
  *used = type == 2 ? (1ull << 30) : env_mib("MOCKSMI_USED_MIB", 5000);
  return 0;
}
struct vram_usage { uint32_t total, used, reserved[2]; };
EXPORT int amdsmi_get_gpu_vram_usage(void* h, vram_usage* u) {
  if (h != (void*)1 || !u) return 2;
  u->total = (uint32_t)(env_mib("MOCKSMI_TOTAL_MIB", 294912) >> 20);
  u->used = (uint32_t)(env_mib("MOCKSMI_USED_MIB", 5000) >> 20);
  return 0;
}
struct vram_info { int type; char vendor[256]; uint64_t size; uint32_t width; uint64_t bw; uint64_t reserved[37]; };
EXPORT int amdsmi_get_gpu_vram_info(void* h, vram_info* i) {
  if (h != (void*)1 || !i) return 2;
  memset(i, 0, sizeof(*i));
  i->size = env_mib("MOCKSMI_TOTAL_MIB", 294912) >> 20;
  return 0;
}
EXPORT int rsmi_dev_pci_id_get(uint32_t dv, uint64_t* id) {
  if (dv != 0 || !id) return 2;
  unsigned dom, bus, dev, fn;
  bdf_fields(&dom, &bus, &dev, &fn);
  *id = (uint64_t)fn | ((uint64_t)dev << 3) | ((uint64_t)bus << 8) | ((uint64_t)dom << 32);
  return 0;
}
EXPORT int rsmi_dev_memory_total_get(uint32_t dv, int type, uint64_t* total) {
  return amdsmi_get_gpu_memory_total(dv == 0 ? (void*)1 : nullptr, type, total);
}
EXPORT int rsmi_dev_memory_usage_get(uint32_t dv, int type, uint64_t* used) {
  return amdsmi_get_gpu_memory_usage(dv == 0 ? (void*)1 : nullptr, type, used);
}
}
