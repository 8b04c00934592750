#include "http.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>
#include <thread>

#include "json.hpp"
#include "util.hpp"

namespace bee {

static constexpr size_t kMaxHeaderBytes = 64 * 1024;
static constexpr int kMaxConnections = 2048;

const char* http_reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 413: return "Payload Too Large";
    case 422: return "Unprocessable Entity";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
  }
  return "Status";
}

void HttpResponse::error(int code, const std::string& detail) {
  Json j = Json::object();
  j.set("detail", detail);
  json(code, j.dump());
}

// ---- body reader ---------------------------------------------------------------

bool BodyReader::fill(size_t want) {
  while (pending_.size() < want) {
    char buf[1 << 16];
    ssize_t r = recv(fd_, buf, sizeof buf, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    pending_.append(buf, (size_t)r);
  }
  return true;
}

std::string BodyReader::next(size_t max) {
  if (finished_) return "";
  if (!chunked_) {
    if (left_ <= 0) {
      finished_ = true;
      return "";
    }
    if (pending_.empty() && !fill(1)) throw std::runtime_error("connection closed mid-body");
    size_t n = std::min<size_t>({pending_.size(), (size_t)left_, max});
    std::string out = pending_.substr(0, n);
    pending_.erase(0, n);
    left_ -= (int64_t)n;
    if (left_ == 0) finished_ = true;
    return out;
  }
  if (chunk_header_needed_) {
    size_t eol;
    while ((eol = pending_.find("\r\n")) == std::string::npos) {
      if (pending_.size() > 1024 || !fill(pending_.size() + 1)) throw std::runtime_error("bad chunk header");
    }
    std::string line = pending_.substr(0, eol);
    pending_.erase(0, eol + 2);
    // chunk-size = 1*HEXDIG [ ";" ext ]: anything else (a sign, no digits,
    // > 2^60) is a malformed request, not a length
    size_t digits = 0;
    uint64_t size = 0;
    while (digits < line.size() && isxdigit((unsigned char)line[digits])) {
      if (size >> 60) throw std::runtime_error("bad chunk header");
      const char c = line[digits];
      size = size * 16 + (uint64_t)(c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10);
      ++digits;
    }
    if (digits == 0 || (digits < line.size() && line[digits] != ';' && line[digits] != ' ' && line[digits] != '\t'))
      throw std::runtime_error("bad chunk header");
    left_ = (int64_t)size;
    chunk_header_needed_ = false;
    if (left_ == 0) {  // last chunk: skip trailers up to the blank line
      while (true) {
        size_t e;
        while ((e = pending_.find("\r\n")) == std::string::npos) {
          if (!fill(pending_.size() + 1)) throw std::runtime_error("bad chunk trailer");
        }
        std::string t = pending_.substr(0, e);
        pending_.erase(0, e + 2);
        if (t.empty()) break;
      }
      finished_ = true;
      return "";
    }
  }
  if (pending_.empty() && !fill(1)) throw std::runtime_error("connection closed mid-chunk");
  size_t n = std::min<size_t>({pending_.size(), (size_t)left_, max});
  std::string out = pending_.substr(0, n);
  pending_.erase(0, n);
  left_ -= (int64_t)n;
  if (left_ == 0) {
    if (!fill(2)) throw std::runtime_error("bad chunk terminator");
    pending_.erase(0, 2);
    chunk_header_needed_ = true;
  }
  if (out.empty()) return next(max);
  return out;
}

std::string BodyReader::read_all(int64_t limit) {
  std::string out;
  while (true) {
    std::string piece = next();
    if (piece.empty() && finished_) break;
    out += piece;
    if ((int64_t)out.size() > limit) throw std::length_error("body too large");
  }
  return out;
}

bool BodyReader::stream_to_fd(int out_fd, int64_t limit, std::string* err) {
  int64_t total = 0;
  try {
    while (true) {
      std::string piece = next(1 << 20);
      if (piece.empty() && finished_) break;
      total += (int64_t)piece.size();
      if (limit > 0 && total > limit) {
        if (err) *err = "body too large";
        return false;
      }
      if (!write_all(out_fd, piece)) {
        if (err) *err = std::string("write: ") + strerror(errno);
        return false;
      }
    }
  } catch (const std::exception& e) {
    if (err) *err = e.what();
    return false;
  }
  return true;
}

void BodyReader::drain() {
  try {
    while (!finished_) next(1 << 20);
  } catch (...) {
    finished_ = true;
  }
}

// ---- server ---------------------------------------------------------------------

bool HttpServer::listen(const std::string& spec, std::string* err) {
  if (spec.rfind("unix:", 0) == 0) {
    unix_path_ = spec.substr(5);
    listen_fd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_un addr{};
    addr.sun_family = AF_UNIX;
    if (unix_path_.size() >= sizeof addr.sun_path) {
      *err = "unix socket path too long";
      return false;
    }
    strncpy(addr.sun_path, unix_path_.c_str(), sizeof addr.sun_path - 1);
    unlink(unix_path_.c_str());
    if (bind(listen_fd_, (sockaddr*)&addr, sizeof addr) != 0) {
      *err = std::string("bind ") + unix_path_ + ": " + strerror(errno);
      return false;
    }
    chmod(unix_path_.c_str(), 0600);  // the service (same UID) only
    bound_ = spec;
  } else {
    size_t colon = spec.rfind(':');
    std::string host = colon == std::string::npos ? "0.0.0.0" : spec.substr(0, colon);
    std::string port = colon == std::string::npos ? spec : spec.substr(colon + 1);
    if (host.empty() || host == "*") host = "0.0.0.0";
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE;
    int rc = getaddrinfo(host.c_str(), port.c_str(), &hints, &res);
    if (rc != 0 || !res) {
      *err = std::string("getaddrinfo: ") + gai_strerror(rc);
      return false;
    }
    listen_fd_ = socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (bind(listen_fd_, res->ai_addr, res->ai_addrlen) != 0) {
      *err = std::string("bind ") + spec + ": " + strerror(errno);
      freeaddrinfo(res);
      return false;
    }
    freeaddrinfo(res);
    sockaddr_storage ss{};
    socklen_t sl = sizeof ss;
    getsockname(listen_fd_, (sockaddr*)&ss, &sl);
    int bound_port = ss.ss_family == AF_INET6 ? ntohs(((sockaddr_in6*)&ss)->sin6_port) : ntohs(((sockaddr_in*)&ss)->sin_port);
    bound_ = host + ":" + std::to_string(bound_port);
  }
  if (::listen(listen_fd_, 1024) != 0) {
    *err = std::string("listen: ") + strerror(errno);
    return false;
  }
  return true;
}

void HttpServer::stop() {
  stopping_ = true;
  if (listen_fd_ >= 0) shutdown(listen_fd_, SHUT_RDWR);
  if (!unix_path_.empty()) unlink(unix_path_.c_str());
}

void HttpServer::serve_forever() {
  while (!stopping_) {
    int fd = accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      if (stopping_) break;
      if (errno == EMFILE || errno == ENFILE) {
        usleep(10000);
        continue;
      }
      BEE_ERROR("accept: %s", strerror(errno));
      break;
    }
    if (active_.load() >= kMaxConnections) {
      const char* busy = "HTTP/1.1 503 Service Unavailable\r\nContent-Length: 0\r\nConnection: close\r\n\r\n";
      send(fd, busy, strlen(busy), MSG_NOSIGNAL);
      close(fd);
      continue;
    }
    if (!unix_path_.empty() && peer_filter_) {
      ucred cred{};
      socklen_t len = sizeof cred;
      if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cred, &len) != 0 || !peer_filter_(cred.pid, cred.uid)) {
        BEE_WARN("control socket: refused peer pid %d uid %d", (int)cred.pid, (int)cred.uid);
        close(fd);
        continue;
      }
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    active_++;
    std::thread([this, fd] {
      ThreadRoleScope role(kThrHttp);
      handle_conn(fd);
      active_--;
    }).detach();
  }
}

static std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

static bool send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t w = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += (size_t)w;
  }
  return true;
}

void HttpServer::handle_conn(int fd) {
  std::string buf;
  while (!stopping_) {
    // read headers
    size_t hdr_end;
    while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
      if (buf.size() > kMaxHeaderBytes) {
        send_all(fd, "HTTP/1.1 413 Payload Too Large\r\nContent-Length: 0\r\nConnection: close\r\n\r\n");
        close(fd);
        return;
      }
      char tmp[16384];
      ssize_t r = recv(fd, tmp, sizeof tmp, 0);
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) {
        close(fd);
        return;
      }
      buf.append(tmp, (size_t)r);
    }
    std::string head = buf.substr(0, hdr_end);
    buf.erase(0, hdr_end + 4);

    HttpRequest req;
    size_t line_end = head.find("\r\n");
    std::string request_line = head.substr(0, line_end);
    size_t sp1 = request_line.find(' '), sp2 = request_line.rfind(' ');
    if (sp1 == std::string::npos || sp2 == sp1) {
      send_all(fd, "HTTP/1.1 400 Bad Request\r\nContent-Length: 0\r\nConnection: close\r\n\r\n");
      close(fd);
      return;
    }
    req.method = request_line.substr(0, sp1);
    req.target = request_line.substr(sp1 + 1, sp2 - sp1 - 1);
    std::string version = request_line.substr(sp2 + 1);
    size_t pos = line_end == std::string::npos ? head.size() : line_end + 2;
    while (pos < head.size()) {
      size_t e = head.find("\r\n", pos);
      if (e == std::string::npos) e = head.size();
      std::string line = head.substr(pos, e - pos);
      size_t colon = line.find(':');
      if (colon != std::string::npos) {
        std::string v = line.substr(colon + 1);
        size_t a = v.find_first_not_of(" \t");
        size_t b = v.find_last_not_of(" \t");
        req.headers[lower(line.substr(0, colon))] = a == std::string::npos ? "" : v.substr(a, b - a + 1);
      }
      pos = e + 2;
    }
    size_t q = req.target.find('?');
    req.path = url_decode(req.target.substr(0, q));
    if (q != std::string::npos) {
      std::string qs = req.target.substr(q + 1);
      size_t p = 0;
      while (p <= qs.size()) {
        size_t amp = qs.find('&', p);
        if (amp == std::string::npos) amp = qs.size();
        std::string kv = qs.substr(p, amp - p);
        size_t eq = kv.find('=');
        if (!kv.empty()) req.query[url_decode(kv.substr(0, eq))] = eq == std::string::npos ? "" : url_decode(kv.substr(eq + 1));
        p = amp + 1;
      }
    }
    bool chunked = lower(req.header("transfer-encoding")).find("chunked") != std::string::npos;
    int64_t clen = req.header("content-length").empty() ? 0 : strtoll(req.header("content-length").c_str(), nullptr, 10);
    BodyReader body(fd, buf, chunked ? 0 : clen, chunked);
    req.body = &body;
    bool keep_alive = version == "HTTP/1.1" ? lower(req.header("connection")) != "close"
                                             : lower(req.header("connection")) == "keep-alive";

    HttpResponse resp;
    CpuScope cpu(kCpuHttp);
    try {
      handler_(req, resp);
    } catch (const std::exception& e) {
      resp = HttpResponse();
      resp.error(500, std::string("internal error: ") + e.what());
    }
    body.drain();

    int file_fd = -1;
    int64_t file_size = 0;
    if (!resp.file_path.empty()) {
      file_fd = open(resp.file_path.c_str(), O_RDONLY | O_CLOEXEC);
      struct stat st;
      if (file_fd < 0 || fstat(file_fd, &st) != 0 || !S_ISREG(st.st_mode)) {
        if (file_fd >= 0) close(file_fd);
        file_fd = -1;
        resp.error(404, "file not found");
        resp.file_path.clear();
      } else {
        file_size = st.st_size;
      }
    }
    std::string out = "HTTP/1.1 " + std::to_string(resp.status) + " " + http_reason(resp.status) + "\r\n";
    if (resp.status != 204) {
      out += "Content-Type: " + resp.content_type + "\r\n";
      out += "Content-Length: " + std::to_string(file_fd >= 0 ? file_size : (int64_t)resp.body.size()) + "\r\n";
    }
    for (auto& kv : resp.headers) out += kv.first + ": " + kv.second + "\r\n";
    out += keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
    bool ok = send_all(fd, out);
    if (ok && file_fd >= 0) {
      off_t off = 0;
      while (off < file_size) {
        ssize_t n = sendfile(fd, file_fd, &off, (size_t)(file_size - off));
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) {
          ok = false;
          break;
        }
      }
    } else if (ok && resp.status != 204) {
      ok = send_all(fd, resp.body);
    }
    if (file_fd >= 0) close(file_fd);
    if (!ok || !keep_alive) break;
  }
  close(fd);
}

}  // namespace bee
