// Native rendezvous key-value store over TCP (the bootstrap half of SURVEY §5.8: "a small C++
// TCP store on master-ip:6585; rank 0 creates the ncclUniqueId, the others fetch it").
//
// Rank 0 runs the server thread; every rank (including 0) talks to it through a client socket.
// Operations: set(key, bytes), get(key) -> bytes (blocks until present or timeout), add(key, n) ->
// new value (atomic counter), wait(keys), delete(key), and a counter barrier built on add+wait that
// removes its keys when the last participant leaves.  Length-prefixed binary protocol; one request in flight per client.
#pragma once
#include <atomic>
#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dpa {

class TcpStoreServer {
 public:
  TcpStoreServer(const std::string& host, int port);  // binds + listens (port 0 = ephemeral)
  ~TcpStoreServer();
  int port() const { return port_; }

 private:
  void accept_loop();
  void serve(int fd);

  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> stop_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
  std::vector<std::thread> workers_;
  std::vector<int> client_fds_;
};

class TcpStoreClient {
 public:
  TcpStoreClient(const std::string& host, int port, double timeout_s);
  ~TcpStoreClient();
  void set(const std::string& key, const std::string& value);
  // blocks until the key exists, at most timeout_s (< 0: the client's default timeout)
  std::string get(const std::string& key, double timeout_s = -1.0);
  long long add(const std::string& key, long long delta);
  bool del(const std::string& key);  // true if the key existed
  long long num_keys();
  void wait(const std::vector<std::string>& keys, double timeout_s = -1.0);
  // all `world` participants call with the same tag; returns once all arrived; its keys are
  // deleted by the last participant to leave
  void barrier(const std::string& tag, int world);

 private:
  std::string request(char op, const std::string& key, const std::string& value);

  int fd_ = -1;
  double timeout_s_;
  std::mutex mu_;
};

}  // namespace dpa
