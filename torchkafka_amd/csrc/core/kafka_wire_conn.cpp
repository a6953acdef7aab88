// Native Kafka wire-protocol client, transport: one broker connection (TCP, TLS through OpenSSL,
// SASL PLAIN / SCRAM-SHA-256/512 / OAUTHBEARER, ApiVersions negotiation, request framing and
// the incremental response reader).  The requests built on it are in kafka_wire.cpp; see
// kafka_wire.h.
#include "kafka_wire.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/rand.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>

namespace tk::wire {

// ------------------------------------------------------------ Conn
namespace {
int64_t mono_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000 + ts.tv_nsec / 1000000;
}
}  // namespace

// OpenSSL's latest error, for exceptions (also used by Client's TLS context setup)
std::string ssl_error(const std::string& what) {
  char buf[256];
  const unsigned long e = ERR_get_error();
  ERR_error_string_n(e, buf, sizeof(buf));
  return what + ": " + (e ? std::string(buf) : std::string("TLS failure"));
}

Conn::Conn(const std::string& host, int port, int timeout_ms, const Security* sec, SSL_CTX* ctx)
    : host_(host), port_(port), timeout_ms_(timeout_ms), buf_(size_t(1) << 16) {
  open_socket(sec, ctx);
  negotiate(sec, ctx);
  if (sec && sec->sasl()) authenticate(*sec);
}

void Conn::open_socket(const Security* sec, SSL_CTX* ctx) {
  const std::string& host = host_;
  const int port = port_;
  const int timeout_ms = timeout_ms_;
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw KafkaError("NoBrokersAvailable: cannot resolve " + host + ":" + ps);
  std::string why = "no address";
  for (addrinfo* a = res; a; a = a->ai_next) {
    int fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    // non-blocking connect bounded by the timeout
    int fl = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &fl, sizeof(fl));
    int rcv = 8 << 20;
    ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof(rcv));
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    if (::connect(fd, a->ai_addr, a->ai_addrlen) == 0) {
      fd_ = fd;
      break;
    }
    why = std::strerror(errno);
    ::close(fd);
  }
  freeaddrinfo(res);
  if (fd_ < 0) throw KafkaError("NoBrokersAvailable: cannot connect to " + host + ":" + ps + " (" + why + ")");
  if (sec && sec->tls()) {
    if (!ctx) throw KafkaError("wire: TLS requested without a TLS context");
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    ::setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));  // bounds the handshake
    ssl_ = SSL_new(ctx);
    SSL_set_fd(ssl_, fd_);
    SSL_set_tlsext_host_name(ssl_, host.c_str());
    if (sec->check_hostname) {
      X509_VERIFY_PARAM* vp = SSL_get0_param(ssl_);
      X509_VERIFY_PARAM_set_hostflags(vp, X509_CHECK_FLAG_NO_PARTIAL_WILDCARDS);
      X509_VERIFY_PARAM_set1_host(vp, host.c_str(), 0);
    }
    if (SSL_connect(ssl_) != 1) {
      const std::string e = ssl_error("KafkaConnectionError: TLS handshake with " + host + ":" + ps);
      close();
      throw KafkaError(e);
    }
    timeval none{0, 0};
    ::setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
  }
}

// ApiVersions v0 (every broker since 0.10 answers it, before authentication too).  A broker
// that predates it closes the connection: reconnect and use the fixed legacy versions.
void Conn::negotiate(const Security* sec, SSL_CTX* ctx) {
  std::vector<uint8_t> resp;
  try {
    resp = roundtrip(kApiVersions, 0, "torchkafka", std::string(), timeout_ms_);
  } catch (const KafkaError&) {
    close();
    b0_ = b1_ = 0;
    remaining_ = 0;
    open_socket(sec, ctx);
    broker_.clear();
    return;
  }
  Reader r(resp.data(), resp.size());
  const int16_t e = r.i16();
  const int32_t n = r.i32();
  std::map<int16_t, ApiRange> m;
  for (int32_t i = 0; i < n; ++i) {
    const int16_t key = r.i16();
    const int16_t lo = r.i16();
    const int16_t hi = r.i16();
    m[key] = ApiRange{lo, hi};
  }
  if (e != kNone && m.empty()) {
    close();
    throw WireError(e, std::string(error_name(e)) + ": ApiVersions refused by " + host_);
  }
  broker_ = std::move(m);
}

int16_t Conn::version(int16_t api_key) const {
  if (broker_.empty()) return legacy_version(api_key);
  const auto& cv = client_versions();
  auto c = cv.find(api_key);
  auto b = broker_.find(api_key);
  if (c == cv.end() || b == broker_.end())
    throw WireError(kUnsupportedVersion, "UnsupportedVersionError: " + host_ + " does not serve API " +
                                             std::to_string(api_key));
  const int16_t hi = std::min(c->second.max, b->second.max);
  const int16_t lo = std::max(c->second.min, b->second.min);
  if (hi < lo)
    throw WireError(kUnsupportedVersion,
                    "UnsupportedVersionError: API " + std::to_string(api_key) + ": " + host_ + " serves v" +
                        std::to_string(b->second.min) + "-" + std::to_string(b->second.max) + ", this client v" +
                        std::to_string(c->second.min) + "-" + std::to_string(c->second.max));
  return hi;
}

namespace {

std::string b64(const std::string& s) {
  std::string out(4 * ((s.size() + 2) / 3) + 1, '\0');
  const int n = EVP_EncodeBlock(reinterpret_cast<unsigned char*>(&out[0]),
                                reinterpret_cast<const unsigned char*>(s.data()), int(s.size()));
  out.resize(size_t(n));
  return out;
}

std::string unb64(const std::string& s) {
  if (s.size() % 4) throw KafkaError("SaslAuthenticationFailedError: bad base64 from the server");
  std::string out(s.size() / 4 * 3 + 1, '\0');
  const int n = EVP_DecodeBlock(reinterpret_cast<unsigned char*>(&out[0]),
                                reinterpret_cast<const unsigned char*>(s.data()), int(s.size()));
  if (n < 0) throw KafkaError("SaslAuthenticationFailedError: bad base64 from the server");
  size_t pad = 0;
  for (size_t i = s.size(); i > 0 && s[i - 1] == '='; --i) ++pad;
  out.resize(size_t(n) - pad);
  return out;
}

std::string hmac(const EVP_MD* md, const std::string& key, const std::string& msg) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned len = 0;
  HMAC(md, key.data(), int(key.size()), reinterpret_cast<const unsigned char*>(msg.data()), msg.size(), out, &len);
  return std::string(reinterpret_cast<char*>(out), len);
}

std::string digest(const EVP_MD* md, const std::string& msg) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned len = 0;
  EVP_Digest(msg.data(), msg.size(), out, &len, md, nullptr);
  return std::string(reinterpret_cast<char*>(out), len);
}

// "a=1,b=2" -> value of `key`
std::string scram_attr(const std::string& msg, char key) {
  size_t i = 0;
  while (i < msg.size()) {
    size_t j = msg.find(',', i);
    if (j == std::string::npos) j = msg.size();
    if (j - i >= 2 && msg[i] == key && msg[i + 1] == '=') return msg.substr(i + 2, j - i - 2);
    i = j + 1;
  }
  return "";
}

}  // namespace

// One SaslAuthenticate v0 round: sends `token`, returns the server's bytes (throws on an error).
std::string Conn::sasl_round(const std::string& token) {
  Writer au;
  au.i32(int32_t(token.size()));
  au.data().append(token);
  const int16_t v = version(kSaslAuthenticate);
  auto r = roundtrip(kSaslAuthenticate, v, "torchkafka", au.data(), timeout_ms_);
  Reader b(r.data(), r.size());
  const int16_t e = b.i16();
  const std::string msg = b.str();
  int32_t len = 0;
  const uint8_t* p = b.bytes(&len);
  if (v >= 1) b.i64();  // session lifetime (KIP-368): re-authentication is not needed here
  if (e != kNone) {
    close();
    throw KafkaError("SaslAuthenticationFailedError: " + (msg.empty() ? std::string(error_name(e)) : msg));
  }
  return len > 0 ? std::string(reinterpret_cast<const char*>(p), size_t(len)) : std::string();
}

// SCRAM-SHA-256 / SCRAM-SHA-512 (RFC 5802 / 7677): two SaslAuthenticate rounds; the server's
// signature is checked too, so a man in the middle without the password is detected.
void Conn::scram(const Security& sec) {
  const EVP_MD* md = sec.sasl_mechanism == "SCRAM-SHA-512" ? EVP_sha512() : EVP_sha256();
  unsigned char rnd[24];
  if (RAND_bytes(rnd, sizeof(rnd)) != 1) throw KafkaError("SASL: no random bytes for the SCRAM nonce");
  const std::string cnonce = b64(std::string(reinterpret_cast<char*>(rnd), sizeof(rnd)));
  std::string user;
  for (char ch : sec.username) user += ch == '=' ? "=3D" : ch == ',' ? "=2C" : std::string(1, ch);
  const std::string first_bare = "n=" + user + ",r=" + cnonce;
  const std::string server_first = sasl_round("n,," + first_bare);
  const std::string nonce = scram_attr(server_first, 'r'), salt = unb64(scram_attr(server_first, 's'));
  const int iters = std::atoi(scram_attr(server_first, 'i').c_str());
  if (nonce.compare(0, cnonce.size(), cnonce) != 0 || iters < 1) {
    close();
    throw KafkaError("SaslAuthenticationFailedError: malformed SCRAM server-first message");
  }
  const int hlen = EVP_MD_get_size(md);
  std::string salted(size_t(hlen), '\0');
  PKCS5_PBKDF2_HMAC(sec.password.data(), int(sec.password.size()), reinterpret_cast<const unsigned char*>(salt.data()),
                    int(salt.size()), iters, md, hlen, reinterpret_cast<unsigned char*>(&salted[0]));
  const std::string client_key = hmac(md, salted, "Client Key");
  const std::string stored_key = digest(md, client_key);
  const std::string final_wo_proof = "c=biws,r=" + nonce;  // biws = base64("n,,")
  const std::string auth_msg = first_bare + "," + server_first + "," + final_wo_proof;
  std::string proof = hmac(md, stored_key, auth_msg);
  for (size_t i = 0; i < proof.size(); ++i) proof[i] = char(proof[i] ^ client_key[i]);
  const std::string server_final = sasl_round(final_wo_proof + ",p=" + b64(proof));
  const std::string expect = b64(hmac(md, hmac(md, salted, "Server Key"), auth_msg));
  if (scram_attr(server_final, 'v') != expect) {
    close();
    throw KafkaError("SaslAuthenticationFailedError: the server's SCRAM signature does not match");
  }
}

// OAUTHBEARER (RFC 7628 section 3.1): one client message -- the GS2 header "n,," then
// 0x01-separated "auth=Bearer <token>" and the extensions, closed by 0x01 0x01.  A server that
// rejects the token answers with an error challenge (JSON); the client acknowledges it with a
// lone 0x01 (section 3.2.3) and the exchange fails.
void Conn::oauthbearer(const Security& sec) {
  std::string token, ext;
  if (sec.oauth) {
    std::lock_guard<std::mutex> l(sec.oauth->m);
    token = sec.oauth->token;
    ext = sec.oauth->extensions;
  }
  if (token.empty()) {
    close();
    throw KafkaError("SaslAuthenticationFailedError: OAUTHBEARER needs a token (sasl_oauth_token_provider)");
  }
  std::string msg = std::string("n,,\x01") + "auth=Bearer " + token;  // (a hex escape would eat the 'a')
  if (!ext.empty()) msg += "\x01" + ext;
  msg += "\x01\x01";
  const std::string challenge = sasl_round(msg);
  if (!challenge.empty()) {
    try {
      sasl_round(std::string(1, '\x01'));
    } catch (const KafkaError&) {
    }
    close();
    throw KafkaError("SaslAuthenticationFailedError: OAUTHBEARER token rejected: " + challenge);
  }
}

void Conn::authenticate(const Security& sec) {
  const bool is_scram = sec.sasl_mechanism == "SCRAM-SHA-256" || sec.sasl_mechanism == "SCRAM-SHA-512";
  const bool is_oauth = sec.sasl_mechanism == "OAUTHBEARER";
  if (sec.sasl_mechanism != "PLAIN" && !is_scram && !is_oauth)
    throw KafkaError("UnsupportedSaslMechanismError: " + sec.sasl_mechanism +
                     " (this client speaks PLAIN, SCRAM-SHA-256, SCRAM-SHA-512 and OAUTHBEARER)");
  Writer hs;
  hs.str(sec.sasl_mechanism);
  auto r1 = roundtrip(kSaslHandshake, version(kSaslHandshake), "torchkafka", hs.data(), timeout_ms_);
  Reader a(r1.data(), r1.size());
  const int16_t e1 = a.i16();
  if (e1 != kNone) {
    close();
    throw KafkaError(std::string(error_name(e1)) + ": SaslHandshake " + sec.sasl_mechanism + " refused by " + host_);
  }
  if (is_scram) {
    scram(sec);
    return;
  }
  if (is_oauth) {
    oauthbearer(sec);
    return;
  }
  std::string token;
  token.push_back('\0');
  token += sec.username;
  token.push_back('\0');
  token += sec.password;
  sasl_round(token);
}

ssize_t Conn::io_recv(void* dst, size_t n) {
  if (!ssl_) return ::recv(fd_, dst, n, 0);
  const int k = SSL_read(ssl_, dst, int(std::min<size_t>(n, INT32_MAX)));
  if (k > 0) return k;
  const int err = SSL_get_error(ssl_, k);
  if (err == SSL_ERROR_WANT_READ || err == SSL_ERROR_WANT_WRITE) {
    errno = EAGAIN;
    return -1;
  }
  return k == 0 ? 0 : -1;
}

bool Conn::wait_readable(int ms) {
  if (ssl_ && SSL_pending(ssl_) > 0) return true;  // decrypted bytes already buffered
  pollfd p{fd_, POLLIN, 0};
  const int r = ::poll(&p, 1, ms);
  if (r < 0 && errno != EINTR) {
    close();
    throw KafkaError("KafkaConnectionError: poll failed");
  }
  return r > 0;
}

Conn::~Conn() { close(); }

void Conn::close() {
  if (ssl_) {
    SSL_free(ssl_);
    ssl_ = nullptr;
  }
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

void Conn::send_all(const std::string& frame) {
  size_t off = 0;
  while (off < frame.size()) {
    const ssize_t n = ssl_ ? ssize_t(SSL_write(ssl_, frame.data() + off, int(frame.size() - off)))
                           : ::send(fd_, frame.data() + off, frame.size() - off, MSG_NOSIGNAL);
    if (ssl_ && n <= 0) {
      const std::string e = ssl_error("KafkaConnectionError: TLS send");
      close();
      throw KafkaError(e);
    }
    if (n < 0) {
      if (errno == EINTR) continue;
      const std::string e = std::strerror(errno);
      close();
      throw KafkaError("KafkaConnectionError: send to " + host_ + " failed: " + e);
    }
    off += size_t(n);
  }
}

void Conn::send(int16_t api_key, int16_t api_version, const std::string& client_id, const std::string& body) {
  if (fd_ < 0) throw KafkaError("KafkaConnectionError: connection to " + host_ + " is closed");
  if (remaining_) finish();
  Writer h;
  h.i32(0);  // size, patched below
  h.i16(api_key);
  h.i16(api_version);
  expect_corr_ = ++corr_;
  h.i32(expect_corr_);
  h.str(client_id);
  std::string& f = h.data();
  f.append(body);
  const uint32_t sz = htonl(uint32_t(f.size() - 4));
  std::memcpy(&f[0], &sz, 4);
  send_all(f);
}

void Conn::check_cancel() {
  if (cancel_ && cancel_->load(std::memory_order_relaxed)) {
    close();
    throw KafkaError("KafkaError: request cancelled (client stopping)");
  }
}

void Conn::fill(size_t want) {
  // compact, then read until `want` bytes are buffered (never past the current response)
  if (b0_ == b1_) b0_ = b1_ = 0;
  if (b0_ > 0 && buf_.size() - b1_ < want) {
    std::memmove(buf_.data(), buf_.data() + b0_, b1_ - b0_);
    b1_ -= b0_;
    b0_ = 0;
  }
  if (buf_.size() < want) buf_.resize(want);
  while (b1_ - b0_ < want) {
    const int64_t left = deadline_ms_ - mono_ms();
    if (left <= 0) {
      close();
      throw KafkaError("KafkaTimeoutError: no response from " + host_ + ":" + std::to_string(port_));
    }
    check_cancel();
    if (!wait_readable(int(std::min<int64_t>(left, 100)))) continue;
    const ssize_t n = io_recv(buf_.data() + b1_, buf_.size() - b1_);
    if (n == 0 || (n < 0 && errno != EINTR && errno != EAGAIN)) {
      close();
      throw KafkaError("KafkaConnectionError: connection to " + host_ + " closed by the broker");
    }
    if (n > 0) b1_ += size_t(n);
  }
}

size_t Conn::begin_response(int timeout_ms) {
  remaining_ = 0;
  deadline_ms_ = mono_ms() + timeout_ms;
  fill(8);
  uint32_t sz, corr;
  std::memcpy(&sz, buf_.data() + b0_, 4);
  std::memcpy(&corr, buf_.data() + b0_ + 4, 4);
  b0_ += 8;
  sz = ntohl(sz);
  corr = ntohl(corr);
  if (sz < 4 || int32_t(corr) != expect_corr_) {
    close();
    throw KafkaError("wire: response correlation mismatch from " + host_);
  }
  remaining_ = sz - 4;
  return remaining_;
}

void Conn::read(void* dst, size_t n) {
  if (n > remaining_) throw KafkaError("wire: read past the end of a response");
  if (b1_ - b0_ < n && n <= 4096) fill(n);  // small fields: one recv fills the buffer for many of them
  auto* d = static_cast<uint8_t*>(dst);
  const size_t have = std::min(n, b1_ - b0_);
  std::memcpy(d, buf_.data() + b0_, have);
  b0_ += have;
  size_t off = have;
  // large reads go straight from the socket into the destination (record sets into the log)
  while (off < n) {
    const int64_t left = deadline_ms_ - mono_ms();
    if (left <= 0) {
      close();
      throw KafkaError("KafkaTimeoutError: response from " + host_ + " stalled");
    }
    check_cancel();
    if (!wait_readable(int(std::min<int64_t>(left, 100)))) continue;
    const ssize_t got = io_recv(d + off, n - off);
    if (got == 0 || (got < 0 && errno != EINTR && errno != EAGAIN)) {
      close();
      throw KafkaError("KafkaConnectionError: connection to " + host_ + " closed mid-response");
    }
    if (got > 0) off += size_t(got);
  }
  remaining_ -= n;
}

int8_t Conn::r8() { int8_t v; read(&v, 1); return v; }
int16_t Conn::r16() { uint16_t v; read(&v, 2); return int16_t(ntohs(v)); }
int32_t Conn::r32() { uint32_t v; read(&v, 4); return int32_t(ntohl(v)); }
int64_t Conn::r64() {
  const uint64_t hi = uint32_t(r32());
  const uint64_t lo = uint32_t(r32());
  return int64_t((hi << 32) | lo);
}
std::string Conn::rstr() {
  const int16_t n = r16();
  if (n <= 0) return std::string();
  std::string s(size_t(n), '\0');
  read(&s[0], size_t(n));
  return s;
}
void Conn::skip(size_t n) {
  uint8_t tmp[4096];
  while (n) {
    const size_t k = std::min(n, sizeof(tmp));
    read(tmp, k);
    n -= k;
  }
}
void Conn::finish() { skip(remaining_); }

std::vector<uint8_t> Conn::roundtrip(int16_t api_key, int16_t api_version, const std::string& client_id,
                                     const std::string& body, int timeout_ms) {
  send(api_key, api_version, client_id, body);
  const size_t n = begin_response(timeout_ms);
  std::vector<uint8_t> out(n);
  read(out.data(), n);
  return out;
}

}  // namespace tk::wire
