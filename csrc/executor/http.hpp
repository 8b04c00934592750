// Small HTTP/1.1 server: thread per connection, keep-alive, Content-Length
// and chunked request bodies (httpx streams uploads chunked), file responses
// via sendfile.  Listens on TCP ("host:port") or a Unix socket ("unix:/path").
#pragma once
#include <atomic>
#include <functional>
#include <map>
#include <string>
#include <vector>

namespace bee {

class BodyReader {
 public:
  BodyReader(int fd, std::string& pending, int64_t content_length, bool chunked)
      : fd_(fd), pending_(pending), left_(content_length), chunked_(chunked) {}
  // next piece of body (empty = end); throws std::runtime_error on I/O errors
  std::string next(size_t max = 1 << 16);
  std::string read_all(int64_t limit);  // throws if body > limit
  bool stream_to_fd(int out_fd, int64_t limit, std::string* err);
  void drain();
  bool done() const { return finished_; }

 private:
  bool fill(size_t want);
  int fd_;
  std::string& pending_;
  int64_t left_;  // content-length mode: bytes left; chunked: bytes left in chunk
  bool chunked_;
  bool finished_ = false;
  bool chunk_header_needed_ = true;
};

struct HttpRequest {
  std::string method;
  std::string target;  // raw target incl. query
  std::string path;    // url-decoded path without query
  std::map<std::string, std::string> query;
  std::map<std::string, std::string> headers;  // lower-case keys
  BodyReader* body = nullptr;
  std::string header(const std::string& k) const {
    auto it = headers.find(k);
    return it == headers.end() ? "" : it->second;
  }
};

struct HttpResponse {
  int status = 200;
  std::string content_type = "application/json";
  std::string body;
  std::string file_path;  // if set, stream this file as the body
  std::map<std::string, std::string> headers;
  void json(int code, const std::string& text) {
    status = code;
    content_type = "application/json";
    body = text;
  }
  void error(int code, const std::string& detail);
};

using HttpHandler = std::function<void(HttpRequest&, HttpResponse&)>;

class HttpServer {
 public:
  explicit HttpServer(HttpHandler h) : handler_(std::move(h)) {}
  bool listen(const std::string& spec, std::string* err);  // "host:port" | "unix:/path"
  void serve_forever();                                    // blocks
  void stop();
  std::string bound_address() const { return bound_; }
  // Unix-socket listeners: refuse peers for which this returns false
  // (called with the peer's pid/uid from SO_PEERCRED before any byte is read)
  void set_peer_filter(std::function<bool(pid_t, uid_t)> f) { peer_filter_ = std::move(f); }

 private:
  void handle_conn(int fd);
  HttpHandler handler_;
  std::function<bool(pid_t, uid_t)> peer_filter_;
  int listen_fd_ = -1;
  std::string bound_;
  std::string unix_path_;
  std::atomic<bool> stopping_{false};
  std::atomic<int> active_{0};
};

const char* http_reason(int code);

}  // namespace bee
