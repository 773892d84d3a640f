// glibc ABI floor of libmivgpu.so (force-included into the shim build).
//
// The shim is preloaded into every process of a tenant container, whatever
// distribution the image is built on.  Built as is on Ubuntu 22.04 it needed
// GLIBC_2.34 (pthread_*, dl* moved into libc), GLIBC_2.33 (stat/fstat) and a
// shared libstdc++ with GLIBCXX_3.4.29: on a RHEL/UBI 8 (glibc 2.28) or
// Ubuntu 20.04 (2.31) image ld.so printed "cannot be preloaded: ignored" and
// the pod ran with no limit at all.
//
// Every libc import is therefore bound to the OLDEST version glibc exports it
// under (all <= GLIBC_2.17, the floor asserted by tests/test_shim_abi_floor.py);
// glibc >= 2.34 still exports those versions as compatibility symbols, and
// on older glibc they are the default versions of libpthread.so.0 / libdl.so.2,
// which the link names as NEEDED (utils/build.py).  libstdc++ and libgcc are
// linked statically and hidden by the version script.  (Sanitizer builds,
// which need the runtime's interceptors on the current versions, leave
// MIVGPU_GLIBC_FLOOR undefined and get plain stat/fstat.)
#ifndef MIVGPU_GLIBC_FLOOR_H
#define MIVGPU_GLIBC_FLOOR_H

#if defined(__x86_64__) && defined(MIVGPU_GLIBC_FLOOR)
__asm__(".symver dlopen,dlopen@GLIBC_2.2.5");
__asm__(".symver dlerror,dlerror@GLIBC_2.2.5");
__asm__(".symver dladdr,dladdr@GLIBC_2.2.5");
__asm__(".symver pthread_create,pthread_create@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_init,pthread_mutexattr_init@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_destroy,pthread_mutexattr_destroy@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_setpshared,pthread_mutexattr_setpshared@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_setrobust,pthread_mutexattr_setrobust@GLIBC_2.12");
__asm__(".symver pthread_mutex_consistent,pthread_mutex_consistent@GLIBC_2.12");
__asm__(".symver pthread_key_create,pthread_key_create@GLIBC_2.2.5");
__asm__(".symver pthread_getspecific,pthread_getspecific@GLIBC_2.2.5");
__asm__(".symver pthread_setspecific,pthread_setspecific@GLIBC_2.2.5");
__asm__(".symver pthread_key_delete,pthread_key_delete@GLIBC_2.2.5");
__asm__(".symver pthread_attr_init,pthread_attr_init@GLIBC_2.2.5");
__asm__(".symver pthread_attr_destroy,pthread_attr_destroy@GLIBC_2.2.5");
__asm__(".symver pthread_attr_setdetachstate,pthread_attr_setdetachstate@GLIBC_2.2.5");
__asm__(".symver __xstat,__xstat@GLIBC_2.2.5");
__asm__(".symver __fxstat,__fxstat@GLIBC_2.2.5");
// The statically linked libstdc++ objects (gthr) hold WEAK references to
// pthread_once and __pthread_key_create that no .symver of ours can reach:
// the shim defines both itself (hidden), forwarding to these old versions.
__asm__(".symver mivgpu_glibc_pthread_once,pthread_once@GLIBC_2.2.5");
__asm__(".symver mivgpu_glibc_pthread_key_create,__pthread_key_create@GLIBC_2.2.5");
#endif

#ifdef __cplusplus
#include <pthread.h>
#include <sys/stat.h>
#if defined(__x86_64__) && defined(MIVGPU_GLIBC_FLOOR)
extern "C" {
// stat/fstat became real functions (GLIBC_2.33); before that they were inline
// wrappers over these (struct stat layout unchanged on x86-64, _STAT_VER 1).
int __xstat(int ver, const char* path, struct stat* st);
int __fxstat(int ver, int fd, struct stat* st);
int mivgpu_glibc_pthread_once(pthread_once_t* once, void (*init)(void));
int mivgpu_glibc_pthread_key_create(pthread_key_t* key, void (*dtor)(void*));
}
static inline int mivgpu_stat(const char* path, struct stat* st) { return __xstat(1, path, st); }
static inline int mivgpu_fstat(int fd, struct stat* st) { return __fxstat(1, fd, st); }
#else  // sanitizer builds: the runtime must intercept the current versions
static inline int mivgpu_stat(const char* path, struct stat* st) { return stat(path, st); }
static inline int mivgpu_fstat(int fd, struct stat* st) { return fstat(fd, st); }
#endif
#endif

#endif  // MIVGPU_GLIBC_FLOOR_H
