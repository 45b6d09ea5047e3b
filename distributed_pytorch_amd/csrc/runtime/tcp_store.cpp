#include "tcp_store.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>

namespace dpa {

namespace {

enum : char { OP_SET = 'S', OP_GET = 'G', OP_ADD = 'A', OP_DEL = 'D', OP_NKEYS = 'N' };
enum : char { ST_OK = 0, ST_TIMEOUT = 1 };

bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool send_blob(int fd, const std::string& s) {
  const uint32_t n = htonl((uint32_t)s.size());
  return send_all(fd, &n, 4) && send_all(fd, s.data(), s.size());
}

bool recv_blob(int fd, std::string& s) {
  uint32_t n = 0;
  if (!recv_all(fd, &n, 4)) return false;
  n = ntohl(n);
  if (n > (64u << 20)) return false;  // sanity bound: values are ids / counters
  s.resize(n);
  return n == 0 || recv_all(fd, &s[0], n);
}

std::string i64(long long v) { return std::string(reinterpret_cast<const char*>(&v), 8); }
long long i64of(const std::string& s) {
  long long v = 0;
  if (s.size() == 8) std::memcpy(&v, s.data(), 8);
  return v;
}

}  // namespace

// ------------------------------------------------------------------ server
TcpStoreServer::TcpStoreServer(const std::string& host, int port) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("TcpStore: socket() failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (host.empty() || host == "0.0.0.0") {
    a.sin_addr.s_addr = htonl(INADDR_ANY);
  } else if (::inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    ::close(listen_fd_);
    throw std::runtime_error("TcpStore: server host must be an IPv4 address: " + host);
  }
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(listen_fd_, 256) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("TcpStore: cannot bind/listen on " + host + ":" + std::to_string(port));
  }
  socklen_t len = sizeof(a);
  ::getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&a), &len);
  port_ = ntohs(a.sin_port);
  acceptor_ = std::thread([this] { accept_loop(); });
}

TcpStoreServer::~TcpStoreServer() {
  stop_ = true;
  ::shutdown(listen_fd_, SHUT_RDWR);
  ::close(listen_fd_);
  if (acceptor_.joinable()) acceptor_.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    // SHUT_RD only: a reply being written completes; a worker blocked in recv sees EOF and exits
    for (int fd : client_fds_) ::shutdown(fd, SHUT_RD);
  }
  cv_.notify_all();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  for (int fd : client_fds_) ::close(fd);
}

void TcpStoreServer::accept_loop() {
  while (!stop_) {
    const int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) {
      if (stop_) return;
      continue;
    }
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(mu_);
    client_fds_.push_back(fd);
    workers_.emplace_back([this, fd] { serve(fd); });
  }
}

void TcpStoreServer::serve(int fd) {
  while (!stop_) {
    char op = 0;
    std::string key, val;
    if (!recv_all(fd, &op, 1) || !recv_blob(fd, key) || !recv_blob(fd, val)) return;
    char st = ST_OK;
    std::string out;
    if (op == OP_SET) {
      std::lock_guard<std::mutex> g(mu_);
      kv_[key] = val;
      cv_.notify_all();
    } else if (op == OP_ADD) {
      std::lock_guard<std::mutex> g(mu_);
      const long long v = i64of(kv_[key]) + i64of(val);
      kv_[key] = i64(v);
      out = i64(v);
      cv_.notify_all();
    } else if (op == OP_GET) {  // val = timeout in ms (decimal)
      const long ms = std::strtol(val.c_str(), nullptr, 10);
      std::unique_lock<std::mutex> lk(mu_);
      const bool ok = cv_.wait_for(lk, std::chrono::milliseconds(ms),
                                   [&] { return stop_.load() || kv_.count(key) > 0; });
      if (ok && kv_.count(key)) {
        out = kv_[key];
      } else {
        st = ST_TIMEOUT;
      }
    } else if (op == OP_DEL) {
      std::lock_guard<std::mutex> g(mu_);
      out = i64(kv_.erase(key) ? 1 : 0);
    } else if (op == OP_NKEYS) {
      std::lock_guard<std::mutex> g(mu_);
      out = i64((long long)kv_.size());
    } else {
      return;  // protocol error: drop the connection
    }
    if (!send_all(fd, &st, 1) || !send_blob(fd, out)) return;
  }
}

// ------------------------------------------------------------------ client
TcpStoreClient::TcpStoreClient(const std::string& host, int port, double timeout_s) : timeout_s_(timeout_s) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("TcpStore: cannot resolve " + host);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  // the server may not be up yet: retry until the deadline
  while (true) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd_ >= 0 && ::connect(fd_, res->ai_addr, res->ai_addrlen) == 0) break;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    if (std::chrono::steady_clock::now() > deadline) {
      ::freeaddrinfo(res);
      throw std::runtime_error("TcpStore: cannot connect to " + host + ":" + std::to_string(port));
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  ::freeaddrinfo(res);
  int one = 1;
  ::setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

TcpStoreClient::~TcpStoreClient() {
  if (fd_ >= 0) ::close(fd_);
}

std::string TcpStoreClient::request(char op, const std::string& key, const std::string& value) {
  std::lock_guard<std::mutex> g(mu_);
  if (!send_all(fd_, &op, 1) || !send_blob(fd_, key) || !send_blob(fd_, value))
    throw std::runtime_error("TcpStore: connection lost (send)");
  char st = 0;
  std::string out;
  if (!recv_all(fd_, &st, 1) || !recv_blob(fd_, out)) throw std::runtime_error("TcpStore: connection lost (recv)");
  if (st == ST_TIMEOUT) throw std::runtime_error("TcpStore: timed out waiting for key '" + key + "'");
  return out;
}

void TcpStoreClient::set(const std::string& key, const std::string& value) { request(OP_SET, key, value); }

std::string TcpStoreClient::get(const std::string& key, double timeout_s) {
  const double t = timeout_s >= 0 ? timeout_s : timeout_s_;
  return request(OP_GET, key, std::to_string((long)(t * 1000.0)));
}

long long TcpStoreClient::add(const std::string& key, long long delta) { return i64of(request(OP_ADD, key, i64(delta))); }

bool TcpStoreClient::del(const std::string& key) { return i64of(request(OP_DEL, key, "")) != 0; }

long long TcpStoreClient::num_keys() { return i64of(request(OP_NKEYS, "", "")); }

// every key within ONE overall deadline (not timeout_s per key)
void TcpStoreClient::wait(const std::vector<std::string>& keys, double timeout_s) {
  const double t = timeout_s >= 0 ? timeout_s : timeout_s_;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(t);
  for (const auto& k : keys) {
    const double left = std::chrono::duration<double>(deadline - std::chrono::steady_clock::now()).count();
    get(k, left > 0 ? left : 0.0);
  }
}

// Counter barrier that leaves nothing behind: arrivals count up, the last arrival publishes
// "done", every rank then checks out, and the last to check out deletes the three keys (nobody
// reads them any more).
void TcpStoreClient::barrier(const std::string& tag, int world) {
  const std::string cnt = "__barrier_cnt/" + tag, done = "__barrier_done/" + tag, out = "__barrier_out/" + tag;
  const long long n = add(cnt, 1);
  if (n == world) set(done, "1");
  get(done);
  if (add(out, 1) == world) {
    del(cnt);
    del(done);
    del(out);
  }
}

}  // namespace dpa
