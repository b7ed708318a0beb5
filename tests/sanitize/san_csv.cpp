// Sanitizer harness (test infrastructure, CPU only) for the product path's host CSV code
// (trajectory_generation_amd/csrc/dataset_csv.cpp: traj_dataset_write_csv / _csv_rows / _read_csv), built with
// -fsanitize=address,undefined by tests/test_sanitizers.py: multi-threaded write and read of tricky values
// (signed zeros, subnormals, 1e16 boundary, huge, NaN, inf), thread counts above the row count, and degenerate or
// malformed files (empty, header only, no final newline, CRLF, short / long / garbage rows, wrong row counts).
// Every round trip must be exact and every malformed file an error or a defined result -- never a read past a buffer.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/trajmpc.h"

static int fails = 0;
#define CHECK(cond)                                                   \
    do {                                                              \
        if (!(cond)) {                                                \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

static void write_file(const std::string& p, const std::string& s) {
    FILE* f = std::fopen(p.c_str(), "wb");
    std::fwrite(s.data(), 1, s.size(), f);
    std::fclose(f);
}

static bool same(double a, double b) {
    return (std::isnan(a) && std::isnan(b)) || (a == b && std::signbit(a) == std::signbit(b));
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : ".";
    unsigned long long s = 0x9e3779b97f4a7c15ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (double)(s >> 11) / 9007199254740992.0; };
    const double special[] = {0.0, -0.0, 5e-324, -2.5e-310, 1e16, 9999999999999998.0, 1e-5, 0.0001, 123456.0,
                              1.7976931348623157e308, -1e300, 0.1, 1.0 / 3.0};
    for (int B : {0, 1, 7}) {
        for (int T : {0, 1, 13}) {
            const int R = T + 1;
            std::vector<double> X((size_t)B * R * 6), U((size_t)B * T * 2), W((size_t)B * R * 6);
            std::vector<long long> ids(B);
            for (int b = 0; b < B; ++b) ids[b] = 1000 + 3 * b;
            for (size_t i = 0; i < X.size(); ++i) X[i] = (i % 5 == 0) ? special[i % 13] : (rnd() - 0.5) * 1e3;
            for (size_t i = 0; i < U.size(); ++i) U[i] = (i % 4 == 0) ? special[(i / 4) % 13] : rnd() - 0.5;
            for (size_t i = 0; i < W.size(); ++i) W[i] = 0.01 * (rnd() - 0.5);
            for (int nt : {1, 3, 64}) {
                const std::string c = dir + "/c.csv", n = dir + "/n.csv";
                CHECK(traj_dataset_write_csv(c.c_str(), n.c_str(), B, T, 0.05, X.data(), U.data(), W.data(), ids.data(),
                                             nt) == TRAJ_OK);
                int nc = 0;
                const long long rows = traj_dataset_csv_rows(c.c_str(), &nc);
                CHECK(rows == (long long)B * R && nc == 10);
                std::vector<double> out((size_t)(rows > 0 ? rows : 1) * 10);
                for (int rt : {1, 4, 200}) {
                    CHECK(traj_dataset_read_csv(c.c_str(), rows, 10, out.data(), rt) == TRAJ_OK);
                    for (int b = 0; b < B; ++b)
                        for (int r = 0; r < R; ++r) {
                            const double* o = out.data() + ((size_t)b * R + r) * 10;
                            for (int k = 0; k < 6; ++k) CHECK(same(o[1 + k], X[((size_t)b * R + r) * 6 + k]));
                            for (int k = 0; k < 2; ++k)
                                CHECK(same(o[7 + k], r < T ? U[((size_t)b * T + r) * 2 + k] : NAN));
                            CHECK(o[9] == (double)ids[b]);
                        }
                    // asking for the wrong row count is an error, not a read past the line table
                    if (rows > 0) CHECK(traj_dataset_read_csv(c.c_str(), rows - 1, 10, out.data(), rt) == TRAJ_E_ARG);
                }
                CHECK(traj_dataset_csv_rows(n.c_str(), &nc) == (long long)B * R && nc == 9);
            }
        }
    }
    // argument errors
    CHECK(traj_dataset_write_csv(nullptr, nullptr, 1, 1, 0.05, nullptr, nullptr, nullptr, nullptr, 1) == TRAJ_E_ARG);
    CHECK(traj_dataset_read_csv(nullptr, 0, 3, nullptr, 1) == TRAJ_E_ARG);
    CHECK(traj_dataset_csv_rows((dir + "/missing.csv").c_str(), nullptr) == TRAJ_E_ARG);
    // degenerate and malformed files
    struct Case { const char* name; const char* body; long long rows; int ncols; int expect; };
    const Case cases[] = {
        {"empty", "", 0, 3, TRAJ_OK},
        {"hdr_nonl", "X,Y,phi", 0, 3, TRAJ_OK},
        {"hdr_only", "X,Y,phi\n", 0, 3, TRAJ_OK},
        {"no_final_nl", "X,Y,phi\n1,2,3\n4,5,6", 2, 3, TRAJ_OK},
        {"crlf", "X,Y,phi\r\n1,2,3\r\n4,5,6\r\n", 2, 3, TRAJ_OK},
        {"empty_fields", "X,Y,phi\n,,\n1,,3\n", 2, 3, TRAJ_OK},
        {"nan_inf", "X,Y,phi\nnan,inf,-inf\nNaN,1e308,-0.0\n", 2, 3, TRAJ_OK},
        {"short_row", "X,Y,phi\n1,2\n", 1, 3, TRAJ_E_ARG},
        {"garbage", "X,Y,phi\n1,zz,3\n", 1, 3, TRAJ_E_ARG},
        {"trailing_garbage", "X,Y,phi\n1,2,3x\n", 1, 3, TRAJ_E_ARG},
        {"blank_line", "X,Y,phi\n1,2,3\n\n4,5,6\n", 3, 3, TRAJ_E_ARG},
        {"huge_token", "X,Y,phi\n1e999999,2,3\n", 1, 3, TRAJ_OK},
    };
    for (const Case& k : cases) {
        const std::string p = dir + "/" + k.name + ".csv";
        write_file(p, k.body);
        int nc = 0;
        const long long rows = traj_dataset_csv_rows(p.c_str(), &nc);
        CHECK(rows == k.rows);
        std::vector<double> out((size_t)(k.rows > 0 ? k.rows : 1) * k.ncols, -7.0);
        for (int rt : {1, 5}) {
            const int e = traj_dataset_read_csv(p.c_str(), k.rows, k.ncols, k.rows ? out.data() : nullptr, rt);
            if (e != k.expect) std::fprintf(stderr, "case %s: %d (expected %d)\n", k.name, e, k.expect);
            CHECK(e == k.expect);
        }
        CHECK(traj_dataset_read_csv(p.c_str(), k.rows + 1, k.ncols, out.data(), 2) == TRAJ_E_ARG);
    }
    std::printf("san_csv %s (%d failed checks)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
