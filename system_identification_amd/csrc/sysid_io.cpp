// sysid_io.cpp — native reader of the reference's .dat logs (ingest).
//
// Format (demo/spot_identification.py:9-14, README.md:50-79): text, one channel per line, one time sample
// per column, tab-delimited.  The reference reads each file with np.loadtxt(..., delimiter='\t',
// dtype=np.float32): every field is converted to double (correctly rounded) and then rounded to float32.
// The fast path below and std::from_chars are correctly rounded too, so the double -> float32 result is
// bit-identical.
//
// The file is read into memory; line boundaries are found with memchr, every line is cut into one byte
// span per thread at tab boundaries, fields are counted per span in parallel (prefix sums give each
// span's first column) and then parsed in parallel.  Decimal fields take Clinger's exact fast path.
#include <algorithm>
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sysid.h"

namespace {

thread_local std::string g_io_error;

int io_err(int code, const std::string& msg) {
  g_io_error = msg;
  return code;
}

bool read_file(const char* path, std::string* buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (n < 0) {
    std::fclose(f);
    return false;
  }
  buf->resize((size_t)n);
  const size_t got = n ? std::fread(&(*buf)[0], 1, (size_t)n, f) : 0;
  std::fclose(f);
  return got == (size_t)n;
}

struct Line {
  const char* b;
  const char* e;
};

// Non-empty lines (np.loadtxt skips blank lines); a trailing '\r' is dropped.
std::vector<Line> split_lines(const std::string& s) {
  std::vector<Line> out;
  const char* p = s.data();
  const char* end = p + s.size();
  while (p < end) {
    const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
    const char* le = nl ? nl : end;
    const char* te = le;
    if (te > p && te[-1] == '\r') --te;
    bool blank = true;
    for (const char* c = p; c < te; ++c)
      if (*c != ' ' && *c != '\t') {
        blank = false;
        break;
      }
    if (!blank) out.push_back({p, te});
    p = nl ? nl + 1 : end;
  }
  return out;
}

int64_t count_fields(const Line& l) {
  int64_t n = 1;
  for (const char* c = l.b; c < l.e; ++c) n += *c == '\t';
  return n;
}

// Clinger's fast path: a decimal with at most 19 significant digits whose value is m * 10^e with
// m < 2^53 and |e| <= 22 is m (exact) times or divided by 10^|e| (exact), one correctly rounded IEEE
// operation.  Covers everything np.savetxt('%.9g') writes; anything else goes to std::from_chars.
bool parse_fast(const char* p, const char* e, double* out) {
  static const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
  uint64_t m = 0;
  int nd = 0, ex = 0;
  bool any = false;
  while (p < e && *p >= '0' && *p <= '9') {
    any = true;
    if (m || *p != '0') {
      if (++nd > 19) return false;
      m = m * 10 + (uint64_t)(*p - '0');
    }
    ++p;
  }
  if (p < e && *p == '.') {
    ++p;
    while (p < e && *p >= '0' && *p <= '9') {
      any = true;
      if (m || *p != '0') {
        if (++nd > 19) return false;
        m = m * 10 + (uint64_t)(*p - '0');
      }
      --ex;
      ++p;
    }
  }
  if (!any) return false;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '-' || *p == '+')) eneg = *p++ == '-';
    if (p == e) return false;
    int x = 0;
    while (p < e && *p >= '0' && *p <= '9') {
      if (x < 10000) x = x * 10 + (*p - '0');
      ++p;
    }
    ex += eneg ? -x : x;
  }
  if (p != e) return false;
  if (m == 0) {
    *out = neg ? -0.0 : 0.0;
    return true;
  }
  if (m >> 53 || ex < -22 || ex > 22) return false;
  const double v = ex < 0 ? (double)m / p10[-ex] : (double)m * p10[ex];
  *out = neg ? -v : v;
  return true;
}

// Parse fields [first, first + count) of a line that starts at `b` (b points at field `first`).
bool parse_span(const char* b, const char* e, int64_t count, float* out) {
  const char* p = b;
  for (int64_t k = 0; k < count; ++k) {
    while (p < e && *p == ' ') ++p;
    const char* q = static_cast<const char*>(std::memchr(p, '\t', (size_t)(e - p)));
    const char* fe = q ? q : e;
    const char* te = fe;
    while (te > p && te[-1] == ' ') --te;
    double v = 0.0;
    const char* s = p;
    if (s < te && *s == '+') ++s;  // from_chars rejects a leading '+', Python's float() accepts it
    if (parse_fast(p, te, &v)) {
      out[k] = (float)v;
      p = q ? q + 1 : e;
      continue;
    }
    const auto r = std::from_chars(s, te, v);
    if (r.ec == std::errc::result_out_of_range && r.ptr == te) {
      // overflow / underflow: Python's float() gives +-inf / +-0 (strtod's HUGE_VAL / 0 with ERANGE)
      std::string f(p, te);
      v = std::strtod(f.c_str(), nullptr);
    } else if (r.ec != std::errc() || r.ptr != te) {
      // inf / nan spellings accepted by np.loadtxt
      std::string f(p, te);
      std::transform(f.begin(), f.end(), f.begin(), [](unsigned char c) { return (char)std::tolower(c); });
      if (f == "nan" || f == "+nan" || f == "-nan") v = __builtin_nan("");
      else if (f == "inf" || f == "+inf" || f == "infinity") v = __builtin_inf();
      else if (f == "-inf" || f == "-infinity") v = -__builtin_inf();
      else return false;
    }
    out[k] = (float)v;
    p = q ? q + 1 : e;
  }
  return true;
}

}  // namespace

extern "C" {

const char* sysid_io_last_error(void) { return g_io_error.c_str(); }

int32_t sysid_dat_shape(const char* path, int64_t* rows, int64_t* cols) {
  if (!path || !rows || !cols) return io_err(SYSID_E_INVALID, "null argument");
  std::string buf;
  if (!read_file(path, &buf)) return io_err(SYSID_E_INVALID, std::string("cannot read ") + path);
  const std::vector<Line> lines = split_lines(buf);
  *rows = (int64_t)lines.size();
  *cols = lines.empty() ? 0 : count_fields(lines[0]);  // the other rows are checked by sysid_dat_read
  return SYSID_OK;
}

int32_t sysid_dat_read(const char* path, float* out, int64_t rows, int64_t cols, int32_t nthreads) {
  if (!path || (!out && rows * cols > 0) || rows < 0 || cols < 0) return io_err(SYSID_E_INVALID, "bad arguments");
  std::string buf;
  if (!read_file(path, &buf)) return io_err(SYSID_E_INVALID, std::string("cannot read ") + path);
  const std::vector<Line> lines = split_lines(buf);
  if ((int64_t)lines.size() != rows) return io_err(SYSID_E_INVALID, std::string(path) + ": row count changed");
  const int T = std::max(1, std::min<int>(nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency(), 64));
  // every line cut into T byte spans that start right after a tab (or at the line start)
  struct Span {
    int64_t row;
    const char* b;
    const char* e;
    int64_t nfield, first;
  };
  std::vector<Span> spans;
  spans.reserve((size_t)rows * T);
  for (int64_t r = 0; r < rows; ++r) {
    const Line& l = lines[(size_t)r];
    const int64_t len = l.e - l.b;
    const char* prev = l.b;
    for (int t = 0; t < T; ++t) {
      const char* e = l.e;
      if (t + 1 < T) {
        const char* x = l.b + len * (t + 1) / T;
        if (x < prev) x = prev;
        const char* q = x < l.e ? static_cast<const char*>(std::memchr(x, '\t', (size_t)(l.e - x))) : nullptr;
        e = q ? q + 1 : l.e;
      }
      if (e > prev || (t == 0 && e == prev)) spans.push_back({r, prev, e, 0, 0});
      prev = e;
      if (prev >= l.e) break;
    }
  }
  auto run = [&](auto&& fn) {
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t)
      pool.emplace_back([&, t] {
        for (size_t i = (size_t)t; i < spans.size(); i += (size_t)T) fn(spans[i]);
      });
    for (size_t i = 0; i < spans.size(); i += (size_t)T) fn(spans[i]);
    for (auto& th : pool) th.join();
  };
  // pass 1: fields per span (a span ends right after a tab, except the line's last one)
  run([&](Span& sp) {
    int64_t n = 0;
    for (const char* c = sp.b; c < sp.e; ++c) n += *c == '\t';
    const Line& l = lines[(size_t)sp.row];
    sp.nfield = sp.e == l.e ? n + 1 : n;
  });
  // field offsets within each line; every row must have `cols` fields
  for (size_t i = 0; i < spans.size();) {
    int64_t f = 0;
    const int64_t r = spans[i].row;
    for (; i < spans.size() && spans[i].row == r; ++i) {
      spans[i].first = f;
      f += spans[i].nfield;
    }
    if (f != cols) return io_err(SYSID_E_INVALID, std::string(path) + ": row " + std::to_string(r) + " has " +
                                                      std::to_string(f) + " columns, expected " + std::to_string(cols));
  }
  // pass 2: parse
  std::vector<char> ok(spans.size(), 1);
  const Span* base = spans.data();
  run([&](Span& sp) {
    const Line& l = lines[(size_t)sp.row];
    ok[(size_t)(&sp - base)] = parse_span(sp.b, l.e, sp.nfield, out + sp.row * cols + sp.first) ? 1 : 0;
  });
  for (size_t i = 0; i < spans.size(); ++i)
    if (!ok[i])
      return io_err(SYSID_E_INVALID, std::string(path) + ": unparsable field in row " + std::to_string(spans[i].row));
  return SYSID_OK;
}

}  // extern "C"
