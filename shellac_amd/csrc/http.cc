// Incremental HTTP/1.1 parser + serializer (see http.h for parity notes).
#include "http.h"

#include <algorithm>
#include <cctype>
#include <cstring>

namespace shellac {

std::string to_lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

static std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) --b;
  return s.substr(a, b - a);
}

std::string canonical_header(const std::string& lower) {
  std::string out = lower;
  bool up = true;
  for (auto& c : out) {
    c = up ? (char)std::toupper((unsigned char)c) : (char)std::tolower((unsigned char)c);
    up = (c == '-');
  }
  return out;
}

std::string gzip_compress(const std::string& in, int level) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, level, Z_DEFLATED, 31, 8, Z_DEFAULT_STRATEGY) != Z_OK) return {};
  std::string out;
  out.resize(deflateBound(&zs, in.size()) + 32);
  zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
  zs.avail_in = (uInt)in.size();
  zs.next_out = reinterpret_cast<Bytef*>(&out[0]);
  zs.avail_out = (uInt)out.size();
  deflate(&zs, Z_FINISH);
  out.resize(zs.total_out);
  deflateEnd(&zs);
  return out;
}

bool gzip_decompress(const std::string& in, std::string* out, uint64_t max_out) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, 31) != Z_OK) return false;
  zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
  zs.avail_in = (uInt)in.size();
  char buf[16384];
  int rc = Z_OK;
  while (rc == Z_OK) {
    zs.next_out = reinterpret_cast<Bytef*>(buf);
    zs.avail_out = sizeof buf;
    rc = inflate(&zs, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) break;
    out->append(buf, sizeof buf - zs.avail_out);
    if (out->size() > max_out) {  // decompression bomb: give up, never allocate past the cap
      rc = Z_MEM_ERROR;
      break;
    }
  }
  inflateEnd(&zs);
  return rc == Z_STREAM_END;
}

HttpParser::HttpParser(bool decode_gzip) : decode_gzip_(decode_gzip) {}

HttpParser::~HttpParser() {
  if (zs_) {
    inflateEnd(zs_);
    delete zs_;
  }
}

void HttpParser::reset() {
  const bool dg = decode_gzip_, eb = eof_body_;
  const size_t mh = max_header_bytes_;
  const uint64_t md = max_decoded_bytes_;
  if (zs_) {
    inflateEnd(zs_);
    delete zs_;
    zs_ = nullptr;
  }
  state_ = kFirstLine;
  decode_gzip_ = dg;
  eof_body_ = eb;
  no_body_ = false;
  max_header_bytes_ = mh;
  max_decoded_bytes_ = md;
  header_bytes_ = 0;
  line_.clear();
  err_.clear();
  is_request_ = true;
  method_.clear(); url_.clear(); reason_.clear();
  status_ = 0; vmaj_ = 1; vmin_ = 1;
  headers_.clear();
  body_.clear();
  chunked_ = gzip_ = false;
  content_length_ = -1;
  remaining_ = 0;
}

void HttpParser::fail(const std::string& m) {
  state_ = kError;
  err_ = m;
}

const std::string* HttpParser::header(const std::string& name) const {
  for (const auto& h : headers_)
    if (h.first == name) return &h.second;
  return nullptr;
}

void HttpParser::set_header(const std::string& name, const std::string& value) {
  remove_header(name);
  headers_.emplace_back(name, value);
}

void HttpParser::remove_header(const std::string& name) {
  headers_.erase(std::remove_if(headers_.begin(), headers_.end(),
                                [&](const Header& h) { return h.first == name; }),
                 headers_.end());
}

bool HttpParser::keep_alive() const {
  const std::string* c = header("connection");
  std::string v = c ? to_lower(*c) : std::string();
  if (v.find("close") != std::string::npos) return false;
  if (v.find("keep-alive") != std::string::npos) return true;
  return vmaj_ > 1 || (vmaj_ == 1 && vmin_ >= 1);
}

std::pair<int, int> HttpParser::keep_alive_params() const {
  if (!keep_alive()) return {0, 1};
  int timeout = 5, maxr = 100;
  const std::string* ka = header("keep-alive");
  if (ka) {
    std::string s = to_lower(*ka);
    size_t i = 0;
    while (i < s.size()) {
      size_t j = s.find(',', i);
      if (j == std::string::npos) j = s.size();
      std::string part = trim(s.substr(i, j - i));
      size_t eq = part.find('=');
      if (eq != std::string::npos) {
        std::string k = trim(part.substr(0, eq)), v = trim(part.substr(eq + 1));
        char* endp = nullptr;
        long n = std::strtol(v.c_str(), &endp, 10);
        if (endp && endp != v.c_str()) {
          if (k == "timeout") timeout = (int)n;
          else if (k == "max") maxr = (int)n;
        }
      }
      i = j + 1;
    }
  }
  return {timeout, maxr};
}

bool HttpParser::take_line(const char*& p, const char* end, std::string* line, size_t* consumed) {
  const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
  if (!nl) {
    line_.append(p, (size_t)(end - p));
    *consumed += (size_t)(end - p);
    p = end;
    return false;
  }
  line_.append(p, (size_t)(nl - p));
  *consumed += (size_t)(nl - p) + 1;
  p = nl + 1;
  if (!line_.empty() && line_.back() == '\r') line_.pop_back();
  line->swap(line_);
  line_.clear();
  return true;
}

bool HttpParser::on_first_line(const std::string& line) {
  if (line.empty()) return true;  // tolerate leading CRLF between pipelined messages
  const size_t s1 = line.find(' ');
  if (s1 == std::string::npos) { fail("malformed start line"); return false; }
  const std::string a = line.substr(0, s1);
  std::string rest = line.substr(s1 + 1);
  auto parse_ver = [&](const std::string& v) -> bool {
    if (v.size() < 8 || v.compare(0, 5, "HTTP/") != 0) return false;
    vmaj_ = v[5] - '0';
    vmin_ = (v.size() > 7 && v[6] == '.') ? v[7] - '0' : 0;
    return vmaj_ >= 0 && vmaj_ <= 9 && vmin_ >= 0 && vmin_ <= 9;
  };
  if (a.compare(0, 5, "HTTP/") == 0) {
    is_request_ = false;
    if (!parse_ver(a)) { fail("bad version"); return false; }
    const size_t s2 = rest.find(' ');
    const std::string code = s2 == std::string::npos ? rest : rest.substr(0, s2);
    reason_ = s2 == std::string::npos ? std::string() : rest.substr(s2 + 1);
    char* endp = nullptr;
    status_ = (int)std::strtol(code.c_str(), &endp, 10);
    if (code.size() != 3 || endp != code.c_str() + 3) { fail("bad status"); return false; }
  } else {
    is_request_ = true;
    const size_t s2 = rest.rfind(' ');
    if (s2 == std::string::npos) { fail("malformed request line"); return false; }
    method_ = a;
    url_ = rest.substr(0, s2);
    if (!parse_ver(rest.substr(s2 + 1))) { fail("bad version"); return false; }
  }
  state_ = kHeaders;
  return true;
}

bool HttpParser::on_header_line(const std::string& line) {
  if (line.empty()) return on_headers_done();
  if ((line[0] == ' ' || line[0] == '\t') && !headers_.empty()) {  // obs-fold
    headers_.back().second += " " + trim(line);
    return true;
  }
  const size_t c = line.find(':');
  if (c == std::string::npos || c == 0) { fail("malformed header"); return false; }
  headers_.emplace_back(to_lower(trim(line.substr(0, c))), trim(line.substr(c + 1)));
  return true;
}

// Comma-separated list elements of every `name` header, trimmed and lower-cased
// (empty elements dropped, RFC 7230 §7).
static std::vector<std::string> header_list(const std::vector<Header>& hs, const char* name) {
  std::vector<std::string> out;
  for (const auto& h : hs) {
    if (h.first != name) continue;
    size_t i = 0;
    const std::string& v = h.second;
    while (i <= v.size()) {
      size_t j = v.find(',', i);
      if (j == std::string::npos) j = v.size();
      std::string t = to_lower(trim(v.substr(i, j - i)));
      if (!t.empty()) out.push_back(std::move(t));
      i = j + 1;
    }
  }
  return out;
}

bool HttpParser::on_headers_done() {
  // Message framing is where a reverse proxy must be strict (RFC 7230 §3.3.3): a
  // request the proxy and the origin could frame differently is a smuggling vector,
  // so anything ambiguous is an error (the proxy answers 400 / treats the upstream
  // as failed) instead of a best guess.
  chunked_ = false;
  bool te_eof = false;  // response: a final coding other than chunked = read to EOF
  const bool has_te = header("transfer-encoding") != nullptr;
  if (has_te) {
    const std::vector<std::string> te = header_list(headers_, "transfer-encoding");
    if (te.empty()) { fail("empty transfer-encoding"); return false; }
    for (size_t i = 0; i < te.size(); ++i) {
      if (te[i] == "chunked" && i + 1 != te.size()) { fail("chunked is not the final coding"); return false; }
      // gzip / deflate / compress transfer-codings are not decoded by this proxy
      if (te[i] != "chunked") { fail("unsupported transfer-coding: " + te[i]); return false; }
    }
    chunked_ = te.back() == "chunked";
    if (!chunked_) {
      if (is_request_) { fail("request transfer-encoding without final chunked"); return false; }
      te_eof = true;
    }
  }
  const std::string* ce = header("content-encoding");
  gzip_ = ce && to_lower(trim(*ce)) == "gzip";
  content_length_ = -1;
  if (header("content-length")) {
    // digits only; repeated values (separate headers or a list) must all agree
    for (const std::string& v : header_list(headers_, "content-length")) {
      if (v.size() > 18 || v.find_first_not_of("0123456789") != std::string::npos) {
        fail("bad content-length");
        return false;
      }
      const int64_t n = (int64_t)std::strtoll(v.c_str(), nullptr, 10);
      if (content_length_ >= 0 && n != content_length_) { fail("conflicting content-length"); return false; }
      content_length_ = n;
    }
    if (content_length_ < 0) { fail("bad content-length"); return false; }
    if (has_te) {
      if (is_request_) { fail("both content-length and transfer-encoding"); return false; }
      content_length_ = -1;  // response: transfer-encoding wins (RFC 7230 §3.3.3 rule 3)
    }
  }
  const bool bodyless_resp =
      !is_request_ && (no_body_ || (status_ >= 100 && status_ < 200) || status_ == 204 ||
                       status_ == 304);
  if (bodyless_resp) {
    state_ = kDone;
  } else if (te_eof) {
    if (!eof_body_) { fail("close-delimited body without eof framing"); return false; }
    state_ = kBodyEof;
  } else if (chunked_) {
    state_ = kChunkSize;
  } else if (content_length_ > 0) {
    remaining_ = (uint64_t)content_length_;
    state_ = kBodyLength;
  } else if (content_length_ == 0 || is_request_) {
    state_ = kDone;
  } else if (eof_body_) {
    state_ = kBodyEof;
  } else {
    state_ = kDone;  // reference parity: unframed response => empty body
  }
  if (state_ == kDone) flush_body();
  return true;
}

void HttpParser::append_body(const char* p, size_t n) {
  if (!n) return;
  if (!(gzip_ && decode_gzip_)) {
    body_.append(p, n);
    return;
  }
  if (!zs_) {
    zs_ = new z_stream;
    std::memset(zs_, 0, sizeof *zs_);
    if (inflateInit2(zs_, 31) != Z_OK) { fail("zlib init"); return; }
  }
  zs_->next_in = reinterpret_cast<Bytef*>(const_cast<char*>(p));
  zs_->avail_in = (uInt)n;
  char buf[16384];
  // until the input is consumed AND inflate stopped filling whole buffers (highly
  // compressible input leaves output pending after its last input byte)
  for (;;) {
    zs_->next_out = reinterpret_cast<Bytef*>(buf);
    zs_->avail_out = sizeof buf;
    const int rc = inflate(zs_, Z_NO_FLUSH);
    body_.append(buf, sizeof buf - zs_->avail_out);
    if (body_.size() > max_decoded_bytes_) { fail("decoded gzip body too large"); return; }
    if (rc == Z_STREAM_END) break;
    if (rc != Z_OK && rc != Z_BUF_ERROR) { fail("bad gzip body"); return; }
    if (zs_->avail_in == 0 && zs_->avail_out != 0) break;
    if (rc == Z_BUF_ERROR && zs_->avail_out != 0) break;
  }
}

void HttpParser::complete_body() {
  flush_body();
  if (state_ != kError) state_ = kDone;
}

void HttpParser::flush_body() {
  if (!zs_ || state_ == kError) return;
  char buf[16384];
  int rc;
  do {
    zs_->next_in = nullptr;
    zs_->avail_in = 0;
    zs_->next_out = reinterpret_cast<Bytef*>(buf);
    zs_->avail_out = sizeof buf;
    rc = inflate(zs_, Z_SYNC_FLUSH);
    body_.append(buf, sizeof buf - zs_->avail_out);
    if (body_.size() > max_decoded_bytes_) { fail("decoded gzip body too large"); return; }
  } while ((rc == Z_OK || rc == Z_BUF_ERROR) && zs_->avail_out == 0);
}

size_t HttpParser::parse(const char* data, size_t len) {
  size_t consumed = 0;
  const char* p = data;
  const char* end = data + len;
  std::string line;
  while (p < end && state_ != kDone && state_ != kError) {
    switch (state_) {
      case kFirstLine:
      case kHeaders:
      case kChunkSize:
      case kChunkCrlf:
      case kTrailers: {
        const size_t before = consumed;
        const bool got = take_line(p, end, &line, &consumed);
        if (state_ == kFirstLine || state_ == kHeaders) {
          header_bytes_ += consumed - before;
          if (header_bytes_ > max_header_bytes_) { fail("header section too large"); break; }
        }
        if (!got) break;
        if (state_ == kFirstLine) {
          on_first_line(line);
        } else if (state_ == kHeaders) {
          on_header_line(line);
        } else if (state_ == kChunkSize) {
          const std::string s = trim(line.substr(0, line.find(';')));
          char* endp = nullptr;
          const unsigned long long n = std::strtoull(s.c_str(), &endp, 16);
          if (s.empty() || *endp != 0) { fail("bad chunk size"); break; }
          if (n == 0) {
            state_ = kTrailers;
          } else {
            remaining_ = n;
            state_ = kChunkData;
          }
        } else if (state_ == kChunkCrlf) {
          if (!line.empty()) { fail("missing CRLF after chunk"); break; }
          state_ = kChunkSize;
        } else {  // trailers: lines until an empty one
          if (line.empty()) complete_body();
        }
        break;
      }
      case kBodyLength:
      case kChunkData: {
        const size_t n = (size_t)std::min<uint64_t>(remaining_, (uint64_t)(end - p));
        append_body(p, n);
        p += n;
        consumed += n;
        remaining_ -= n;
        if (state_ == kError) break;
        if (remaining_ == 0) {
          if (state_ == kBodyLength) {
            complete_body();
          } else {
            state_ = kChunkCrlf;
          }
        }
        break;
      }
      case kBodyEof: {
        append_body(p, (size_t)(end - p));
        consumed += (size_t)(end - p);
        p = end;
        break;
      }
      default:
        break;
    }
  }
  return consumed;
}

bool HttpParser::finish() {
  if (state_ == kBodyEof) complete_body();
  return state_ == kDone;
}

std::string HttpParser::serialize_head(uint64_t body_len, bool with_length) const {
  std::string s;
  s.reserve(256 + headers_.size() * 48);
  char vb[16];
  std::snprintf(vb, sizeof vb, "HTTP/%d.%d", vmaj_, vmin_);
  if (is_request_) {
    s += method_; s += ' '; s += url_; s += ' '; s += vb;
  } else {
    s += vb; s += ' '; s += std::to_string(status_); s += ' '; s += reason_;
  }
  s += "\r\n";
  // join repeats (except Set-Cookie), in first-appearance order
  std::vector<bool> done(headers_.size(), false);
  for (size_t i = 0; i < headers_.size(); ++i) {
    if (done[i]) continue;
    const std::string& k = headers_[i].first;
    if (k == "transfer-encoding" || k == "content-length") continue;
    std::string v = headers_[i].second;
    if (k != "set-cookie") {
      for (size_t j = i + 1; j < headers_.size(); ++j)
        if (!done[j] && headers_[j].first == k) {
          v += ", ";
          v += headers_[j].second;
          done[j] = true;
        }
    }
    s += canonical_header(k); s += ": "; s += v; s += "\r\n";
  }
  const bool bodyless = !is_request_ && ((status_ >= 100 && status_ < 200) || status_ == 204 ||
                                         status_ == 304);
  if (with_length && !bodyless && (body_len > 0 || !is_request_)) {
    s += "Content-Length: ";
    s += std::to_string(body_len);
    s += "\r\n";
  }
  s += "\r\n";
  return s;
}

std::string HttpParser::serialize() const {
  if (gzip_ && decode_gzip_) {
    const std::string z = body_.empty() ? std::string() : gzip_compress(body_, 6);
    return serialize_head(z.size()) + z;
  }
  return serialize_head(body_.size()) + body_;
}

}  // namespace shellac
