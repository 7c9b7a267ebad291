// Standalone check: is hipcub::DeviceRadixSort::SortPairs stable for u64 keys / u32 values?
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
#include <random>
int main() {
  for (int n : {837, 5000, 100000}) {
    std::vector<uint64_t> k(n); std::vector<uint32_t> v(n);
    std::mt19937_64 r(n);
    for (int i = 0; i < n; ++i) { k[i] = r() % 16; v[i] = i; }
    uint64_t *dk, *dk2; uint32_t *dv, *dv2; void* tmp = nullptr; size_t tb = 0;
    hipMalloc(&dk, n*8); hipMalloc(&dk2, n*8); hipMalloc(&dv, n*4); hipMalloc(&dv2, n*4);
    hipMemcpy(dk, k.data(), n*8, hipMemcpyHostToDevice); hipMemcpy(dv, v.data(), n*4, hipMemcpyHostToDevice);
    hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dk2, dv, dv2, n, 0, 64, 0);
    hipMalloc(&tmp, tb);
    hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dk2, dv, dv2, n, 0, 64, 0);
    std::vector<uint64_t> ko(n); std::vector<uint32_t> vo(n);
    hipMemcpy(ko.data(), dk2, n*8, hipMemcpyDeviceToHost); hipMemcpy(vo.data(), dv2, n*4, hipMemcpyDeviceToHost);
    int unsorted = 0, unstable = 0;
    for (int i = 1; i < n; ++i) { if (ko[i] < ko[i-1]) unsorted++; if (ko[i] == ko[i-1] && vo[i] < vo[i-1]) unstable++; }
    printf("n=%d unsorted=%d unstable=%d tmp=%zu\n", n, unsorted, unstable, tb);
  }
  return 0;
}
