// HTTP/2 + gRPC wire helpers shared by the native server (grpc_server.cpp) and
// client (grpc_client.cpp): frame and error codes, the limits both sides
// enforce, frame and gRPC message framing, grpc-message percent coding.
// Internal to src/rpc.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace mi355x::rpc::h2 {

enum FrameType : uint8_t {
  kData = 0,
  kHeaders = 1,
  kPriority = 2,
  kRstStream = 3,
  kSettings = 4,
  kPushPromise = 5,
  kPing = 6,
  kGoaway = 7,
  kWindowUpdate = 8,
  kContinuation = 9,
};
constexpr uint8_t kEndStream = 0x1, kAck = 0x1, kEndHeaders = 0x4, kPadded = 0x8, kPriorityFlag = 0x20;
enum H2Error : uint32_t {
  kNoError = 0,
  kProtocolError = 1,
  kFlowControlError = 3,
  kStreamClosed = 5,
  kFrameSizeError = 6,
  kRefusedStream = 7,
  kCancel = 8,
  kCompressionError = 9,
};

constexpr size_t kOurMaxFrame = 16384;  // SETTINGS_MAX_FRAME_SIZE we accept (the default)
constexpr size_t kMaxHeaderBlock = 64 * 1024;
constexpr size_t kMaxMessage = 4 * 1024 * 1024;
constexpr uint32_t kMaxConcurrentStreams = 128;
constexpr int64_t kMaxWindow = 0x7fffffff;
constexpr char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr size_t kPrefaceLen = 24;

inline uint32_t be32(const uint8_t* p) {
  return (static_cast<uint32_t>(p[0]) << 24) | (static_cast<uint32_t>(p[1]) << 16) |
         (static_cast<uint32_t>(p[2]) << 8) | p[3];
}

inline void put_be32(std::string* out, uint32_t v) {
  out->push_back(static_cast<char>(v >> 24));
  out->push_back(static_cast<char>(v >> 16));
  out->push_back(static_cast<char>(v >> 8));
  out->push_back(static_cast<char>(v));
}

inline void put_frame(std::string* out, uint8_t type, uint8_t flags, uint32_t sid, const char* payload, size_t len) {
  out->push_back(static_cast<char>(len >> 16));
  out->push_back(static_cast<char>(len >> 8));
  out->push_back(static_cast<char>(len));
  out->push_back(static_cast<char>(type));
  out->push_back(static_cast<char>(flags));
  put_be32(out, sid & 0x7fffffffu);
  if (len) out->append(payload, len);
}

inline std::string grpc_frame(const std::string& msg) {
  std::string f;
  f.reserve(5 + msg.size());
  f.push_back('\0');
  put_be32(&f, static_cast<uint32_t>(msg.size()));
  f.append(msg);
  return f;
}

inline std::string percent_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s.substr(0, 1024)) {
    if (c >= 0x20 && c <= 0x7E && c != '%') {
      o.push_back(static_cast<char>(c));
    } else {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    }
  }
  return o;
}

// grpc-message as grpc-go sends it: percent-encoded (a malformed escape is kept as is)
inline std::string percent_decode(const std::string& s) {
  auto hexv = [](char h) {
    return h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10 : h >= 'A' && h <= 'F' ? h - 'A' + 10 : -1;
  };
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && hexv(s[i + 1]) >= 0 && hexv(s[i + 2]) >= 0) {
      o.push_back(static_cast<char>(hexv(s[i + 1]) * 16 + hexv(s[i + 2])));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

inline const char* h2_error_name(uint32_t code) {
  static const char* kNames[] = {"NO_ERROR",      "PROTOCOL_ERROR",     "INTERNAL_ERROR",     "FLOW_CONTROL_ERROR",
                                 "SETTINGS_TIMEOUT", "STREAM_CLOSED",   "FRAME_SIZE_ERROR",   "REFUSED_STREAM",
                                 "CANCEL",        "COMPRESSION_ERROR",  "CONNECT_ERROR",      "ENHANCE_YOUR_CALM",
                                 "INADEQUATE_SECURITY", "HTTP_1_1_REQUIRED"};
  return code < sizeof(kNames) / sizeof(kNames[0]) ? kNames[code] : "UNKNOWN";
}

}  // namespace mi355x::rpc::h2
