// Generates tests/golden/xorwow_rocrand_kat.json from rocRAND's own XORWOW engine
// (host side of /opt/rocm/include/rocrand/rocrand_xorwow.h).  rocRAND and cuRAND
// share the xorwow recurrence and the 2^67-draw subsequence jump; only the
// seeding salts/multipliers and the float mapping differ.  The oracle, run with
// rocRAND's seeding constants, must reproduce these draws (tests/test_xorwow.py).
// Build + run: tests/golden/gen_xorwow_rocrand_kat.sh
#include <rocrand/rocrand_xorwow.h>

#include <cstdio>

int main() {
    const unsigned long long seeds[] = {0ull, 1ull, 1234ull, 0xdeadbeefcafef00dull, 1723000000ull};
    const unsigned long long subs[] = {0ull, 1ull, 2ull, 3ull, 31ull, 32ull, 255ull, 29999ull, 262143ull,
                                       1ull << 24, 123456789ull};
    std::printf("{\"generator\": \"rocrand_device::xorwow_engine (ROCm rocRAND host path)\", \"cases\": [\n");
    bool first = true;
    for (unsigned long long seed : seeds) {
        for (unsigned long long sub : subs) {
            rocrand_device::xorwow_engine e(seed, sub, 0);
            std::printf("%s  {\"seed\": %llu, \"subsequence\": %llu, \"draws\": [", first ? "" : ",\n", seed, sub);
            for (int i = 0; i < 8; ++i) std::printf("%s%u", i ? ", " : "", e.next());
            std::printf("]}");
            first = false;
        }
    }
    std::printf("\n]}\n");
    return 0;
}
