// OAuth2 token sources and request decorators.
//
// Reference: GetTokenSource(ctx, keyFile) returns a JWT token source for a
// service-account key file, or google.DefaultTokenSource with scope
// devstorage.full_control (reference auth.go:28-76); the HTTP client wraps it in
// oauth2.Transport (main.go:83-95) and overrides the User-Agent with "prince"
// (user_agent_round_tripper.go:22-30, main.go:98-101).
#pragma once
#include <memory>
#include <mutex>
#include <string>

#include "http1/http1.h"

namespace gcsb {

constexpr const char* kScopeFullControl = "https://www.googleapis.com/auth/devstorage.full_control";

class TokenSource {
 public:
  virtual ~TokenSource() = default;
  // Current access token (refreshed when within 60 s of expiry).
  virtual std::string token() = 0;
  virtual std::string kind() const = 0;
};

class StaticTokenSource : public TokenSource {
 public:
  explicit StaticTokenSource(std::string t) : tok_(std::move(t)) {}
  std::string token() override { return tok_; }
  std::string kind() const override { return "static"; }

 private:
  std::string tok_;
};

// Base for sources that fetch {access_token, expires_in} from an endpoint.
class CachingTokenSource : public TokenSource {
 public:
  std::string token() override;

 protected:
  // returns token, sets *expires_in_s
  virtual std::string fetch(int64_t* expires_in_s) = 0;

 private:
  std::mutex mu_;
  std::string tok_;
  int64_t expiry_ns_ = 0;
};

// Two-legged JWT flow (RS256 signed with the key file's private key).
class ServiceAccountTokenSource : public CachingTokenSource {
 public:
  // key_json: contents of the service-account JSON; token_uri_override if
  // non-empty replaces the file's token_uri (used against the fake server).
  ServiceAccountTokenSource(const std::string& key_json, std::string scope, std::string token_uri_override = "");
  std::string kind() const override { return "service_account"; }
  std::string build_assertion(int64_t now_s) const;  // exposed for tests

 protected:
  std::string fetch(int64_t* expires_in_s) override;

 private:
  std::string client_email_, private_key_pem_, private_key_id_, token_uri_, scope_;
};

// gcloud "authorized_user" ADC file: refresh-token grant.
class AuthorizedUserTokenSource : public CachingTokenSource {
 public:
  AuthorizedUserTokenSource(const std::string& json, std::string token_uri_override = "");
  std::string kind() const override { return "authorized_user"; }

 protected:
  std::string fetch(int64_t* expires_in_s) override;

 private:
  std::string client_id_, client_secret_, refresh_token_, token_uri_;
};

// GCE metadata server.
class MetadataTokenSource : public CachingTokenSource {
 public:
  explicit MetadataTokenSource(std::string host);  // host[:port]
  std::string kind() const override { return "metadata"; }

 protected:
  std::string fetch(int64_t* expires_in_s) override;

 private:
  std::string host_;
};

// keyFile empty -> application default credentials chain:
// $GOOGLE_APPLICATION_CREDENTIALS, ~/.config/gcloud/application_default_credentials.json,
// then the metadata server ($GCE_METADATA_HOST or 169.254.169.254).
std::shared_ptr<TokenSource> get_token_source(const std::string& key_file, const std::string& scope,
                                              const std::string& token_uri_override = "");

class AuthDecorator : public RequestDecorator {
 public:
  explicit AuthDecorator(std::shared_ptr<TokenSource> ts) : ts_(std::move(ts)) {}
  void decorate(Headers& h) override;

 private:
  std::shared_ptr<TokenSource> ts_;
};

class UserAgentDecorator : public RequestDecorator {
 public:
  explicit UserAgentDecorator(std::string ua) : ua_(std::move(ua)) {}
  void decorate(Headers& h) override { set_header(h, "User-Agent", ua_); }

 private:
  std::string ua_;
};

// RS256 helpers (OpenSSL).
std::string rs256_sign(const std::string& pem_private_key, const std::string& data);
bool rs256_verify(const std::string& pem_public_key, const std::string& data, const std::string& sig);
// Generates a 2048-bit RSA key pair (PEM) — used by tests and the fake server.
void rsa_generate_pem(std::string* private_pem, std::string* public_pem);

}  // namespace gcsb
