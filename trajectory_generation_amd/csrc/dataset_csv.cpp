// dataset_csv.cpp -- host side of the dataset rows: the reference's CSV schema
// written and read natively, multi-threaded.
//
// Writer (generation_type1.py:139-158, :295-339 schema; dataset.write_csv):
//   clean  t,X,Y,phi,vx,vy,omega,d,delta,trajectory_id
//   noisy  t,X,Y,vx,vy,omega,d,delta,trajectory_id          (X..omega + measurement noise, phi dropped)
// one row per time step (T+1 rows per trajectory, t = row * Ts, last row's d / delta NaN).  Floats are
// written the way pandas' to_csv writes a float64 column: the shortest decimal that round-trips (Python
// repr: fixed notation for decimal exponents -4 .. 15 with at least one fractional digit, otherwise
// d.ddde+XX), NaN as an empty field -- the files are byte-identical to the pandas writer's.
//
// Reader (data_loader.py:14-53 input; dataset.load_vehicle_dataset(native=True)): the numeric columns of
// such a file, parsed in parallel chunks with std::from_chars into a caller buffer (row-major [rows, C],
// float64; empty field = NaN), e.g. pinned host memory that is then copied to the device.
#include <algorithm>
#include <atomic>
#include <charconv>
#include <functional>
#include <memory>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/trajmpc.h"

namespace {

// Python repr(float) / numpy str(float64) of a finite double
size_t py_repr(double v, char* out) {
    if (std::isnan(v)) return 0;
    if (std::isinf(v)) {
        const char* s = v < 0 ? "-inf" : "inf";
        std::memcpy(out, s, std::strlen(s));
        return std::strlen(s);
    }
    char sci[64];
    auto r = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific);
    *r.ptr = 0;
    // sci = [-]d[.ddd]e(+|-)XX
    const char* p = sci;
    size_t n = 0;
    if (*p == '-') { out[n++] = '-'; ++p; }
    char dig[32] = {0};
    int nd = 0;
    for (; *p && *p != 'e'; ++p)
        if (*p != '.') dig[nd++] = *p;
    const int e = std::atoi(p + 1);
    if (e >= -4 && e < 16) {
        if (e < 0) {
            out[n++] = '0';
            out[n++] = '.';
            for (int i = 0; i < -e - 1; ++i) out[n++] = '0';
            for (int i = 0; i < nd; ++i) out[n++] = dig[i];
        } else {
            for (int i = 0; i <= e; ++i) out[n++] = i < nd ? dig[i] : '0';
            out[n++] = '.';
            if (nd > e + 1)
                for (int i = e + 1; i < nd; ++i) out[n++] = dig[i];
            else
                out[n++] = '0';
        }
    } else {
        out[n++] = dig[0];
        if (nd > 1) {
            out[n++] = '.';
            for (int i = 1; i < nd; ++i) out[n++] = dig[i];
        }
        out[n++] = 'e';
        out[n++] = e < 0 ? '-' : '+';
        const int ae = e < 0 ? -e : e;
        if (ae < 10) out[n++] = '0';
        auto q = std::to_chars(out + n, out + n + 8, ae);
        n = q.ptr - out;
    }
    return n;
}

void put(std::string& s, double v) {
    char b[48];
    s.append(b, py_repr(v, b));
}

int run_threads(int n, int nthreads, const std::function<void(int, int, int)>& body) {
    nthreads = std::max(1, std::min(nthreads, n));
    std::vector<std::thread> th;
    for (int k = 0; k < nthreads; ++k)
        th.emplace_back(body, k, (int)((long long)n * k / nthreads), (int)((long long)n * (k + 1) / nthreads));
    for (auto& t : th) t.join();
    return nthreads;
}

}  // namespace

extern "C" {

int traj_dataset_write_csv(const char* clean_path, const char* noisy_path, int B, int T, double Ts,
                           const double* X, const double* U, const double* noise, const long long* ids,
                           int nthreads) {
    if (B < 0 || T < 0 || (!clean_path && !noisy_path) || (B > 0 && (!X || (T > 0 && !U) || !ids))) return TRAJ_E_ARG;
    if (noisy_path && B > 0 && !noise) return TRAJ_E_ARG;
    const int R = T + 1;   // rows per trajectory
    for (int which = 0; which < 2; ++which) {
        const char* path = which == 0 ? clean_path : noisy_path;
        if (!path) continue;
        std::vector<std::string> part(std::max(1, std::min(nthreads > 0 ? nthreads : 1, std::max(B, 1))));
        run_threads(B, (int)part.size(), [&](int k, int b0, int b1) {
            std::string& s = part[k];
            s.reserve((size_t)(b1 - b0) * R * 160);
            for (int b = b0; b < b1; ++b) {
                char idb[24];
                const size_t idn = std::to_chars(idb, idb + sizeof(idb), ids[b]).ptr - idb;
                for (int r = 0; r < R; ++r) {
                    const double* x = X + ((size_t)b * R + r) * 6;
                    const double* w = noise ? noise + ((size_t)b * R + r) * 6 : nullptr;
                    put(s, (double)r * Ts);
                    for (int c = 0; c < 6; ++c) {
                        if (which == 1 && c == 2) continue;   // phi is not measured
                        s.push_back(',');
                        put(s, which == 0 ? x[c] : x[c] + w[c]);
                    }
                    for (int c = 0; c < 2; ++c) {
                        s.push_back(',');
                        put(s, r < T ? U[((size_t)b * T + r) * 2 + c] : NAN);
                    }
                    s.push_back(',');
                    s.append(idb, idn);
                    s.push_back('\n');
                }
            }
        });
        FILE* f = std::fopen(path, "wb");
        if (!f) return TRAJ_E_ARG;
        const char* hdr = which == 0 ? "t,X,Y,phi,vx,vy,omega,d,delta,trajectory_id\n"
                                     : "t,X,Y,vx,vy,omega,d,delta,trajectory_id\n";
        bool ok = std::fwrite(hdr, 1, std::strlen(hdr), f) == std::strlen(hdr);
        for (auto& s : part) ok = ok && std::fwrite(s.data(), 1, s.size(), f) == s.size();
        ok = (std::fclose(f) == 0) && ok;
        if (!ok) return TRAJ_E_LAUNCH;
    }
    return TRAJ_OK;
}

long long traj_dataset_csv_rows(const char* path, int* ncols) {
    FILE* f = path ? std::fopen(path, "rb") : nullptr;
    if (!f) return TRAJ_E_ARG;
    std::vector<char> buf(1 << 22);
    long long lines = 0;
    int cols = 1;
    bool header = true;
    char last = '\n';
    size_t n;
    while ((n = std::fread(buf.data(), 1, buf.size(), f)) > 0) {
        const char* p = buf.data();
        const char* end = p + n;
        if (header) {
            const char* nl = (const char*)std::memchr(p, '\n', n);
            for (const char* q = p; q < (nl ? nl : end); ++q) cols += (*q == ',');
            if (!nl) continue;
            header = false;
            p = nl + 1;
        }
        while (p < end && (p = (const char*)std::memchr(p, '\n', end - p)) != nullptr) {
            ++lines;
            ++p;
        }
        last = buf[n - 1];
    }
    std::fclose(f);
    if (!header && last != '\n') ++lines;
    if (ncols) *ncols = cols;
    return lines;
}

int traj_dataset_read_csv(const char* path, long long rows, int ncols, double* out, int nthreads) {
    if (!path || rows < 0 || ncols < 1 || (rows > 0 && !out)) return TRAJ_E_ARG;
    FILE* f = std::fopen(path, "rb");
    if (!f) return TRAJ_E_ARG;
    std::fseek(f, 0, SEEK_END);
    const long size = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (size < 0) {
        std::fclose(f);
        return TRAJ_E_ARG;
    }
    std::unique_ptr<char[]> data(new char[(size_t)size + 1]);   // no zero fill
    const bool rd = std::fread(data.get(), 1, (size_t)size, f) == (size_t)size;
    std::fclose(f);
    if (!rd) return TRAJ_E_LAUNCH;
    data[size] = '\n';
    const char* base = data.get();
    const char* hdr_end = (const char*)std::memchr(base, '\n', (size_t)size + 1);
    const size_t p = (size_t)(hdr_end - base) + 1;
    // an empty file, or a header with no newline (the sentinel's): no data lines at all
    if (p > (size_t)size) return rows == 0 ? TRAJ_OK : TRAJ_E_ARG;
    // line starts after the header, found in parallel chunks (memchr) and concatenated in order
    const int nt = std::max(1, std::min(nthreads > 0 ? nthreads : 1, 64));
    std::vector<std::vector<size_t>> part(nt);
    run_threads(nt, nt, [&](int k, int, int) {
        const size_t c0 = p + ((size_t)size - p) * k / nt, c1 = p + ((size_t)size - p) * (k + 1) / nt;
        auto& v = part[k];
        // a line starts at i if i == p or base[i - 1] == '\n': starts in [c0, c1) come from the newlines
        // at j in [c0 - 1, c1 - 1) (the header's newline at p - 1 is the i == p case)
        if (c0 == p && c0 < c1 && c0 < (size_t)size) v.push_back(c0);
        size_t j = (c0 > p) ? c0 - 1 : p;
        while (j + 1 < c1) {
            const char* nl = (const char*)std::memchr(base + j, '\n', (c1 - 1) - j);
            if (!nl) break;
            const size_t st = (size_t)(nl - base) + 1;
            if (st < (size_t)size) v.push_back(st);
            j = st;
        }
    });
    std::vector<size_t> starts;
    starts.reserve((size_t)rows + 1);
    for (auto& v : part) starts.insert(starts.end(), v.begin(), v.end());
    if ((long long)starts.size() != rows) return TRAJ_E_ARG;
    std::atomic<int> err{0};   // set by any parsing thread
    run_threads((int)rows, nthreads > 0 ? nthreads : 1, [&](int, int r0, int r1) {
        for (int r = r0; r < r1; ++r) {
            const char* s = base + starts[r];
            double* o = out + (size_t)r * ncols;
            for (int c = 0; c < ncols; ++c) {
                const char* e = s;
                while (*e != ',' && *e != '\n' && *e != '\r') ++e;
                if (e == s) {
                    o[c] = NAN;
                } else {
                    auto res = std::from_chars(s, e, o[c]);
                    if (res.ec == std::errc::result_out_of_range && res.ptr == e) {
                        // a literal past the double range: the value Python's float() / pandas give it (+-inf, or a
                        // signed zero / the nearest subnormal), from strtod on the token
                        std::string tok(s, e);
                        o[c] = std::strtod(tok.c_str(), nullptr);
                    } else if (res.ec != std::errc() || res.ptr != e) {
                        // "nan" / "inf" spellings pandas may write
                        std::string tok(s, e);
                        if (tok == "nan" || tok == "NaN") o[c] = NAN;
                        else if (tok == "inf") o[c] = INFINITY;
                        else if (tok == "-inf") o[c] = -INFINITY;
                        else err.store(1, std::memory_order_relaxed);
                    }
                }
                if (c + 1 < ncols) {
                    if (*e != ',') { err.store(1, std::memory_order_relaxed); break; }
                    s = e + 1;
                }
            }
        }
    });
    return err.load() ? TRAJ_E_ARG : TRAJ_OK;
}

}  // extern "C"
