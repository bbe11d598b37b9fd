// Fixture generator for tests/golden/mt_rhs.json: SURVEY §8(d)'s robustness right-hand
// side computed by libstdc++ itself (std::mt19937_64 + std::uniform_real_distribution),
// to pin the oracle's restatement (oracle/pgmg_oracle.c: orc_rhs_mt64) bit for bit.
//   g++ -O2 -std=c++17 -ffp-contract=off tests/golden/make_mt_rhs.cpp -o /tmp/make_mt_rhs
//   /tmp/make_mt_rhs > tests/golden/mt_rhs.json
#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

static uint64_t fnv(const std::vector<double> &v)
{
    uint64_t h = 1469598103934665603ULL;
    for (double d : v) {
        uint64_t w;
        std::memcpy(&w, &d, 8);
        h = (h ^ w) * 1099511628211ULL;
    }
    return h;
}

int main()
{
    std::mt19937_64 d;
    d.discard(9999);
    const uint64_t kat = d();   // [rand.predef]: 9981545732273789042
    std::printf("{\"kat_default_seed_10000th\": \"%" PRIu64 "\", \"fields\": [", kat);
    const int Ns[] = {17, 513, 2049};
    for (int q = 0; q < 3; ++q) {
        const int N = Ns[q];
        std::mt19937_64 g(12345);
        std::uniform_real_distribution<double> u(-1.0, 1.0);
        std::vector<double> f((size_t)N * N);
        for (int j = 0; j < N; ++j)
            for (int i = 0; i < N; ++i) {
                const double v = u(g);
                f[(size_t)j * N + i] = (j == 0 || i == 0 || j == N - 1 || i == N - 1) ? 0.0 : v;
            }
        std::printf("%s{\"N\": %d, \"seed\": 12345, \"hash\": \"%016" PRIx64 "\", \"first_interior\": [", q ? ", " : "",
                    N, fnv(f));
        for (int i = 1; i <= 4; ++i) std::printf("%s%.17g", i > 1 ? ", " : "", f[(size_t)N + i]);
        std::printf("]}");
    }
    std::printf("]}\n");
    return 0;
}
