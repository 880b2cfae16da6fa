// Check of the radix sort call raysort.hip makes (rocprim::radix_sort_pairs on
// 32-bit keys, values = slot indices): the output values must be a permutation
// and the keys ordered in the sorted bits.  Sizes and bit ranges of the batch
// traversal's launches; storage queried for the exact call and, as a second
// case, for a larger element count.
// Finding (ROCm 7.2, gfx950, profiles/r05_rocprim_sort_check.txt): for inputs of
// at most 2^20 elements a bit range with begin_bit > 0 returns neither a
// permutation nor an order (no error code); 2^20 + 1 elements and begin_bit = 0
// are right.  raysort.hip therefore shifts its keys down and sorts [0, bits + 1).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
static bool check(uint32_t n, unsigned begin, unsigned end, bool exact_query, uint32_t seed) {
    std::vector<uint32_t> k(n), v(n);
    std::mt19937 g(seed);
    for (uint32_t i = 0; i < n; i++) { k[i] = g() & 0x7fffffffu; v[i] = i; }
    uint32_t *dk0, *dk1, *dv0, *dv1;
    (void)hipMalloc(&dk0, n * 4); (void)hipMalloc(&dk1, n * 4); (void)hipMalloc(&dv0, n * 4); (void)hipMalloc(&dv1, n * 4);
    (void)hipMemcpy(dk0, k.data(), n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dv0, v.data(), n * 4, hipMemcpyHostToDevice);
    size_t tb = 0;
    const uint32_t qn = exact_query ? n : n + n / 4;
    hipError_t e0 = exact_query ? rocprim::radix_sort_pairs(nullptr, tb, dk0, dk1, dv0, dv1, n, begin, end, 0)
                                : rocprim::radix_sort_pairs(nullptr, tb, dk0, dk1, dv0, dv1, qn, 0u, 32u, 0);
    void* tmp = nullptr;
    (void)hipMalloc(&tmp, tb);
    hipError_t e1 = rocprim::radix_sort_pairs(tmp, tb, dk0, dk1, dv0, dv1, n, begin, end, 0);
    hipError_t e2 = hipDeviceSynchronize();
    std::vector<uint32_t> ko(n), vo(n);
    (void)hipMemcpy(ko.data(), dk1, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(vo.data(), dv1, n * 4, hipMemcpyDeviceToHost);
    std::vector<uint32_t> s = vo;
    std::sort(s.begin(), s.end());
    bool perm = true, ord = true, pairs = true;
    for (uint32_t i = 0; i < n; i++) perm &= s[i] == i;
    const uint32_t mask = end >= 32 ? 0xffffffffu : ((1u << end) - 1u);
    for (uint32_t i = 1; i < n; i++) ord &= ((ko[i - 1] & mask) >> begin) <= ((ko[i] & mask) >> begin);
    for (uint32_t i = 0; i < n; i++) pairs &= vo[i] < n && ko[i] == k[vo[i]];
    std::printf("n %8u bits [%2u,%2u) query %-6s: err %d %d %d temp %9zu perm %d ordered %d pairs %d\n", n, begin, end,
                exact_query ? "exact" : "larger", (int)e0, (int)e1, (int)e2, tb, perm, ord, pairs);
    (void)hipFree(dk0); (void)hipFree(dk1); (void)hipFree(dv0); (void)hipFree(dv1); (void)hipFree(tmp);
    return perm && ord && pairs;
}
int main() {
    int bad = 0;
    for (uint32_t n : {1000u, 65536u, 500000u, 999999u, 1000000u, 1048576u, 1048577u, 2088960u}) {
        for (unsigned begin : {0u, 8u, 19u})
            for (bool exact : {true, false}) bad += !check(n, begin, 32u, exact, n + begin);
        for (unsigned end : {13u, 17u, 25u})   // the workaround: begin 0, keys shifted down
            bad += !check(n, 0u, end, true, n + end) ? 1000 : 0;
    }
    std::printf("%d failing cases of the begin_bit > 0 kind, %d of the [0, end) kind\n", bad % 1000, bad / 1000);
    return 0;
}
