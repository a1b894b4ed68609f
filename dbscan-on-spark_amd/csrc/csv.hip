// csv.hip -- the reference's text I/O around the fit, host code:
//   input   DBSCANSuite.scala:31-33, DBSCANSample.scala:21
//             sc.textFile(path).map(s => Vectors.dense(s.split(',').map(_.toDouble)))
//           one point per line; x = field 0, y = field 1 (DBSCANPoint.scala:23-24 read only
//           vector(0) and vector(1); further fields, e.g. labeled_data.csv's label, are carried
//           but never read); each field parsed as java.lang.Double.parseDouble
//   output  DBSCANSample.scala:35
//             labeledPoints.map(p => s"${p.x},${p.y},${p.cluster}")
//           with java.lang.Double.toString for x and y, as the reference's runtime (JDK 7/8)
//           prints it (jdk8_double_string, javanum.hip).
// Files are memory-mapped and parsed by host threads over newline-aligned byte ranges (count,
// then parse at the counted offsets).
#include "../../include/dbscan_hip.h"
#include "internal.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace dbscan {
namespace {

inline bool java_ws(char c) { return (unsigned char)c <= ' '; }  // String.trim

// java.lang.Double.parseDouble over [b, e): trimmed; optional sign; "NaN", "Infinity", a hex
// floating literal or a decimal one, optionally suffixed by one of f F d D.
bool parse_java_double(const char* b, const char* e, double* out) {
    while (b < e && java_ws(*b)) ++b;
    while (e > b && java_ws(e[-1])) --e;
    if (b == e) return false;
    bool neg = false;
    if (*b == '+' || *b == '-') {
        neg = *b == '-';
        ++b;
    }
    const size_t len = (size_t)(e - b);
    if (len == 3 && memcmp(b, "NaN", 3) == 0) {
        *out = NAN;
        return true;
    }
    if (len == 8 && memcmp(b, "Infinity", 8) == 0) {
        *out = neg ? -INFINITY : INFINITY;
        return true;
    }
    if (len > 0 && (e[-1] == 'f' || e[-1] == 'F' || e[-1] == 'd' || e[-1] == 'D')) --e;
    if (b == e) return false;
    double v = 0;
    if (e - b > 2 && b[0] == '0' && (b[1] == 'x' || b[1] == 'X')) {  // hex: p exponent required
        std::string s(b, e);
        if (s.find_first_of("pP") == std::string::npos) return false;
        char* end = nullptr;
        v = strtod(s.c_str(), &end);
        if (end != s.c_str() + s.size()) return false;
    } else {
        if (!(std::isdigit((unsigned char)*b) || *b == '.')) return false;  // no "inf"/"nan"
        const auto r = std::from_chars(b, e, v, std::chars_format::general);
        if (r.ec == std::errc::result_out_of_range) {  // Java: overflow -> inf, underflow -> 0
            v = strtod(std::string(b, e).c_str(), nullptr);
        } else if (r.ec != std::errc() || r.ptr != e) {
            return false;
        }
    }
    *out = neg ? -v : v;
    return true;
}

struct Mapped {
    const char* data = nullptr;
    size_t size = 0;
    int fd = -1;
    explicit Mapped(const char* path) {
        fd = open(path, O_RDONLY);
        if (fd < 0) throw ArgError{std::string("cannot open ") + path};
        struct stat st;
        void* m = nullptr;
        if (fstat(fd, &st) == 0) {
            size = (size_t)st.st_size;
            m = size > 0 ? mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
        }
        if (m == MAP_FAILED || (size > 0 && !m)) {
            close(fd);
            fd = -1;
            throw ArgError{std::string("cannot map ") + path};
        }
        data = static_cast<const char*>(m);
    }
    ~Mapped() {
        if (data) munmap(const_cast<char*>(data), size);
        if (fd >= 0) close(fd);
    }
};

// Records: the text up to each '\n' (and after the last one, if non-empty -- textFile drops
// only the empty tail after a final newline).
struct Ranges {
    std::vector<size_t> begin;  // per thread: first byte (at a record start)
    std::vector<int64_t> count, first;
};

Ranges split_records(const Mapped& f, int threads) {
    Ranges r;
    const size_t n = f.size;
    r.begin.push_back(0);
    for (int t = 1; t < threads; ++t) {
        size_t at = n * (size_t)t / (size_t)threads;
        if (at <= r.begin.back()) continue;
        const void* nl = memchr(f.data + at, '\n', n - at);
        at = nl ? (size_t)(static_cast<const char*>(nl) - f.data) + 1 : n;
        if (at > r.begin.back() && at < n) r.begin.push_back(at);
    }
    const int T = (int)r.begin.size();
    r.count.assign(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            const size_t b = r.begin[t], e = t + 1 < T ? r.begin[t + 1] : n;
            int64_t c = 0;
            for (size_t i = b; i < e;) {
                const void* nl = memchr(f.data + i, '\n', e - i);
                ++c;
                if (!nl) break;
                i = (size_t)(static_cast<const char*>(nl) - f.data) + 1;
            }
            r.count[t] = c;
        });
    for (auto& x : th) x.join();
    r.first.assign(T, 0);
    for (int t = 1; t < T; ++t) r.first[t] = r.first[t - 1] + r.count[t - 1];
    return r;
}

int host_threads() {
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(h ? h : 1u, 16u));
}

}  // namespace

int64_t csv_read(const char* path, double* x_out, double* y_out, int64_t capacity) {
    Mapped f(path);
    if (f.size == 0) return 0;
    const Ranges r = split_records(f, host_threads());
    const int T = (int)r.begin.size();
    const int64_t total = r.first[T - 1] + r.count[T - 1];
    if (!x_out) return total;
    if (capacity < total) throw ArgError{"dbscan_csv_read: output capacity below the record count"};
    std::vector<int64_t> bad(T, -1);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            const size_t e = t + 1 < T ? r.begin[t + 1] : f.size;
            int64_t k = r.first[t];
            for (size_t i = r.begin[t]; i < e; ++k) {
                const void* nl = memchr(f.data + i, '\n', e - i);
                const size_t le = nl ? (size_t)(static_cast<const char*>(nl) - f.data) : e;
                const char* ls = f.data + i;
                const char* lend = f.data + le;
                while (lend > ls && lend[-1] == ',') --lend;  // split(',') drops trailing empties
                const char* c1 = static_cast<const char*>(memchr(ls, ',', (size_t)(lend - ls)));
                const char* f1e = c1 ? c1 : lend;
                const char* f2b = c1 ? c1 + 1 : lend;
                const char* c2 = c1 ? static_cast<const char*>(memchr(f2b, ',', (size_t)(lend - f2b)))
                                    : nullptr;
                const char* f2e = c2 ? c2 : lend;
                // a line must give two numbers; every further field must still parse (the
                // reference maps each field through toDouble)
                bool ok = c1 && parse_java_double(ls, f1e, &x_out[k]) &&
                          parse_java_double(f2b, f2e, &y_out[k]);
                for (const char* fb = c2; ok && fb; ) {
                    const char* next = static_cast<const char*>(
                        memchr(fb + 1, ',', (size_t)(lend - fb - 1)));
                    double tmp;
                    ok = parse_java_double(fb + 1, next ? next : lend, &tmp);
                    fb = next;
                }
                if (!ok && bad[t] < 0) bad[t] = k;
                i = le + 1;
            }
        });
    for (auto& x : th) x.join();
    for (int t = 0; t < T; ++t)
        if (bad[t] >= 0)
            throw ArgError{"dbscan_csv_read: record " + std::to_string(bad[t] + 1) +
                           " is not x,y[,...] numbers (Double.parseDouble)"};
    return total;
}

void csv_write(const char* path, const double* x, const double* y, const int32_t* cluster,
               int64_t n) {
    FILE* fp = fopen(path, "wb");
    if (!fp) throw ArgError{std::string("cannot create ") + path};
    std::vector<char> buf(1 << 20);
    size_t used = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (used + 128 > buf.size()) {
            fwrite(buf.data(), 1, used, fp);
            used = 0;
        }
        char* p = buf.data() + used;
        p += jdk8_double_string(x[i], p);
        *p++ = ',';
        p += jdk8_double_string(y[i], p);
        p += sprintf(p, ",%d\n", cluster[i]);
        used = (size_t)(p - buf.data());
    }
    const bool ok = fwrite(buf.data(), 1, used, fp) == used;
    if (fclose(fp) != 0 || !ok) throw ArgError{std::string("write failed: ") + path};
}

}  // namespace dbscan
