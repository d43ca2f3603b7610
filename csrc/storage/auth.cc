#include "storage/auth.h"

#include <openssl/bio.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>

#include <chrono>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <thread>

#include "core/util.h"
#include "storage/retry.h"

namespace gcsb {

void sleep_seconds(double s, const volatile bool* cancel) {
  auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(s);
  while (std::chrono::steady_clock::now() < end) {
    if (cancel && *cancel) return;
    auto left = end - std::chrono::steady_clock::now();
    auto step = std::chrono::milliseconds(20);
    std::this_thread::sleep_for(left < step ? left : step);
  }
}

namespace {

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw StorageError("ReadFile(\"" + path + "\"): cannot open", false);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

bool file_exists(const std::string& p) {
  std::ifstream f(p);
  return static_cast<bool>(f);
}

// Split "https://host[:port]/path" into endpoint + path.
void split_uri(const std::string& uri, Endpoint* ep, std::string* path) {
  *ep = Endpoint::parse(uri);
  *path = ep->base_path.empty() ? "/" : ep->base_path;
  ep->base_path.clear();
}

std::string post_form(const std::string& uri, const std::string& form, int64_t* expires_in) {
  Endpoint ep;
  std::string path;
  split_uri(uri, &ep, &path);
  Headers h{{"Content-Type", "application/x-www-form-urlencoded"}};
  SimpleResponse r = http_simple_request(ep, "POST", path, h, form);
  if (r.status != 200)
    throw StorageError("token endpoint " + uri + " returned " + std::to_string(r.status) + ": " + r.body,
                       r.status >= 500 || r.status == 429);
  std::string tok;
  if (!json_get_string(r.body, "access_token", &tok)) throw StorageError("token response without access_token", false);
  int64_t e = 3600;
  json_get_int(r.body, "expires_in", &e);
  *expires_in = e;
  return tok;
}

}  // namespace

std::string CachingTokenSource::token() {
  std::lock_guard<std::mutex> lk(mu_);
  int64_t now = now_ns();
  if (tok_.empty() || now > expiry_ns_ - 60'000'000'000LL) {
    int64_t exp = 3600;
    tok_ = fetch(&exp);
    expiry_ns_ = now + exp * 1'000'000'000LL;
  }
  return tok_;
}

ServiceAccountTokenSource::ServiceAccountTokenSource(const std::string& key_json, std::string scope,
                                                     std::string token_uri_override)
    : scope_(std::move(scope)) {
  std::string type;
  json_get_string(key_json, "type", &type);
  if (!type.empty() && type != "service_account")
    throw StorageError("JWTConfigFromJSON: 'type' field is \"" + type + "\" (expected \"service_account\")", false);
  if (!json_get_string(key_json, "client_email", &client_email_) ||
      !json_get_string(key_json, "private_key", &private_key_pem_))
    throw StorageError("JWTConfigFromJSON: missing client_email/private_key", false);
  json_get_string(key_json, "private_key_id", &private_key_id_);
  if (!json_get_string(key_json, "token_uri", &token_uri_)) token_uri_ = "https://oauth2.googleapis.com/token";
  if (!token_uri_override.empty()) token_uri_ = token_uri_override;
}

std::string ServiceAccountTokenSource::build_assertion(int64_t now_s) const {
  std::string header = "{\"alg\":\"RS256\",\"typ\":\"JWT\"";
  if (!private_key_id_.empty()) header += ",\"kid\":\"" + json_escape(private_key_id_) + "\"";
  header += "}";
  std::string claims = "{\"iss\":\"" + json_escape(client_email_) + "\",\"scope\":\"" + json_escape(scope_) +
                       "\",\"aud\":\"" + json_escape(token_uri_) + "\",\"exp\":" + std::to_string(now_s + 3600) +
                       ",\"iat\":" + std::to_string(now_s) + "}";
  std::string signing_input = base64url_encode(header) + "." + base64url_encode(claims);
  std::string sig = rs256_sign(private_key_pem_, signing_input);
  return signing_input + "." + base64url_encode(sig);
}

std::string ServiceAccountTokenSource::fetch(int64_t* expires_in_s) {
  int64_t now_s = wall_ns() / 1'000'000'000LL;
  std::string form = "grant_type=" + url_encode("urn:ietf:params:oauth:grant-type:jwt-bearer") +
                     "&assertion=" + build_assertion(now_s);
  return post_form(token_uri_, form, expires_in_s);
}

AuthorizedUserTokenSource::AuthorizedUserTokenSource(const std::string& json, std::string token_uri_override) {
  if (!json_get_string(json, "client_id", &client_id_) || !json_get_string(json, "client_secret", &client_secret_) ||
      !json_get_string(json, "refresh_token", &refresh_token_))
    throw StorageError("authorized_user credentials missing fields", false);
  token_uri_ = token_uri_override.empty() ? "https://oauth2.googleapis.com/token" : token_uri_override;
}

std::string AuthorizedUserTokenSource::fetch(int64_t* expires_in_s) {
  std::string form = "grant_type=refresh_token&client_id=" + url_encode(client_id_) +
                     "&client_secret=" + url_encode(client_secret_) + "&refresh_token=" + url_encode(refresh_token_);
  return post_form(token_uri_, form, expires_in_s);
}

MetadataTokenSource::MetadataTokenSource(std::string host) : host_(std::move(host)) {}

std::string MetadataTokenSource::fetch(int64_t* expires_in_s) {
  Endpoint ep = Endpoint::parse("http://" + host_);
  SimpleResponse r = http_simple_request(ep, "GET", "/computeMetadata/v1/instance/service-accounts/default/token",
                                         {{"Metadata-Flavor", "Google"}}, "");
  if (r.status != 200) throw StorageError("metadata server returned " + std::to_string(r.status), r.status >= 500);
  std::string tok;
  if (!json_get_string(r.body, "access_token", &tok)) throw StorageError("metadata token without access_token", false);
  int64_t e = 3600;
  json_get_int(r.body, "expires_in", &e);
  *expires_in_s = e;
  return tok;
}

std::shared_ptr<TokenSource> get_token_source(const std::string& key_file, const std::string& scope,
                                              const std::string& token_uri_override) {
  auto from_file = [&](const std::string& path) -> std::shared_ptr<TokenSource> {
    std::string js = read_file(path);
    std::string type;
    json_get_string(js, "type", &type);
    if (type == "authorized_user") return std::make_shared<AuthorizedUserTokenSource>(js, token_uri_override);
    return std::make_shared<ServiceAccountTokenSource>(js, scope, token_uri_override);
  };
  try {
    if (!key_file.empty()) return from_file(key_file);
    if (const char* env = std::getenv("GOOGLE_APPLICATION_CREDENTIALS"); env && *env) return from_file(env);
    if (const char* home = std::getenv("HOME")) {
      std::string p = std::string(home) + "/.config/gcloud/application_default_credentials.json";
      if (file_exists(p)) return from_file(p);
    }
    const char* mh = std::getenv("GCE_METADATA_HOST");
    return std::make_shared<MetadataTokenSource>(mh && *mh ? mh : "169.254.169.254");
  } catch (const StorageError& e) {
    throw StorageError(std::string(key_file.empty() ? "DefaultTokenSource" : "newTokenSourceFromPath") + ": " +
                           e.what(),
                       false);
  }
}

void AuthDecorator::decorate(Headers& h) { set_header(h, "Authorization", "Bearer " + ts_->token()); }

std::string rs256_sign(const std::string& pem, const std::string& data) {
  BIO* bio = BIO_new_mem_buf(pem.data(), static_cast<int>(pem.size()));
  EVP_PKEY* key = PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  if (!key) throw StorageError("invalid private key PEM", false);
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  size_t siglen = 0;
  std::string sig;
  bool ok = EVP_DigestSignInit(ctx, nullptr, EVP_sha256(), nullptr, key) == 1 &&
            EVP_DigestSignUpdate(ctx, data.data(), data.size()) == 1 &&
            EVP_DigestSignFinal(ctx, nullptr, &siglen) == 1;
  if (ok) {
    sig.resize(siglen);
    ok = EVP_DigestSignFinal(ctx, reinterpret_cast<unsigned char*>(&sig[0]), &siglen) == 1;
    sig.resize(siglen);
  }
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(key);
  if (!ok) throw StorageError("RS256 signing failed", false);
  return sig;
}

bool rs256_verify(const std::string& pem_pub, const std::string& data, const std::string& sig) {
  BIO* bio = BIO_new_mem_buf(pem_pub.data(), static_cast<int>(pem_pub.size()));
  EVP_PKEY* key = PEM_read_bio_PUBKEY(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  if (!key) return false;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  bool ok = EVP_DigestVerifyInit(ctx, nullptr, EVP_sha256(), nullptr, key) == 1 &&
            EVP_DigestVerifyUpdate(ctx, data.data(), data.size()) == 1 &&
            EVP_DigestVerifyFinal(ctx, reinterpret_cast<const unsigned char*>(sig.data()), sig.size()) == 1;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(key);
  return ok;
}

void rsa_generate_pem(std::string* private_pem, std::string* public_pem) {
  EVP_PKEY* key = EVP_RSA_gen(2048);
  if (!key) throw std::runtime_error("RSA keygen failed");
  BIO* b1 = BIO_new(BIO_s_mem());
  PEM_write_bio_PrivateKey(b1, key, nullptr, nullptr, 0, nullptr, nullptr);
  BIO* b2 = BIO_new(BIO_s_mem());
  PEM_write_bio_PUBKEY(b2, key);
  char* p = nullptr;
  long n = BIO_get_mem_data(b1, &p);
  private_pem->assign(p, static_cast<size_t>(n));
  n = BIO_get_mem_data(b2, &p);
  public_pem->assign(p, static_cast<size_t>(n));
  BIO_free(b1);
  BIO_free(b2);
  EVP_PKEY_free(key);
}

}  // namespace gcsb
