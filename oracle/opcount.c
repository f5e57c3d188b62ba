/* oracle/opcount.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Counts the source bytes of every bulk GF(256) op the upstream reference
 * performs, the quantity SURVEY.md section 8(d) defines the algorithmic
 * bytes with.  Linked into _ref/libsiamese_ref_counted.so together with the
 * unmodified reference objects, with
 *   -Wl,--wrap=gf256_add_mem,--wrap=gf256_mul_mem,--wrap=gf256_muladd_mem
 * so every call the codec makes into gf256.cpp (reference gf256.h:244-261;
 * call sites SURVEY.md section 2.2) passes through here first.  Calls gf256.cpp
 * makes to itself are not counted, matching the op-trace definition.
 */
#include <stdint.h>

void __real_gf256_add_mem(void* vx, const void* vy, int bytes);
void __real_gf256_mul_mem(void* vz, const void* vx, uint8_t y, int bytes);
void __real_gf256_muladd_mem(void* vz, uint8_t y, const void* vx, int bytes);

static uint64_t g_bytes;

void __wrap_gf256_add_mem(void* vx, const void* vy, int bytes)
{
    if (bytes > 0)
        __atomic_fetch_add(&g_bytes, (uint64_t)bytes, __ATOMIC_RELAXED);
    __real_gf256_add_mem(vx, vy, bytes);
}

void __wrap_gf256_mul_mem(void* vz, const void* vx, uint8_t y, int bytes)
{
    if (bytes > 0)
        __atomic_fetch_add(&g_bytes, (uint64_t)bytes, __ATOMIC_RELAXED);
    __real_gf256_mul_mem(vz, vx, y, bytes);
}

void __wrap_gf256_muladd_mem(void* vz, uint8_t y, const void* vx, int bytes)
{
    if (bytes > 0)
        __atomic_fetch_add(&g_bytes, (uint64_t)bytes, __ATOMIC_RELAXED);
    __real_gf256_muladd_mem(vz, y, vx, bytes);
}

/* exported for the tests (ctypes) */
__attribute__((visibility("default"))) uint64_t ref_op_bytes(int reset)
{
    const uint64_t v = __atomic_load_n(&g_bytes, __ATOMIC_RELAXED);
    if (reset)
        __atomic_store_n(&g_bytes, 0, __ATOMIC_RELAXED);
    return v;
}
