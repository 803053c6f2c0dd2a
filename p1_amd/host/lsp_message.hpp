// lsp_message.hpp -- C++ mirror of the reference's LSP message type and its
// wire format (the JSON datagrams lspnet carries), for tools and tests that
// speak the miner's protocol framing without the transport itself.
//
//   MsgType / Message / NewConnect / NewData / NewAck / String
//       /root/reference/src/github.com/cmu440/lsp/message.go:8-62
//   Marshal / Unmarshal -- Go encoding/json of Message: fields in declaration
//       order, Payload ([]byte) as standard padded base64, nil as null.
// A bitcoin.Message travels as the Payload of an LSP Data message
// (miner.go:21,55,66: client.Write(json.Marshal(msg))).  The LSP protocol
// itself (epochs, windows, retransmission: SRC/lsp/*_impl.go) is out of scope.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace lsp {

enum MsgType { MsgConnect = 0, MsgData = 1, MsgAck = 2 };  // message.go:8-13

struct Message {  // message.go:16-22
  int64_t Type = MsgConnect;
  int64_t ConnID = 0;
  int64_t SeqNum = 0;
  int64_t Size = 0;
  std::vector<uint8_t> Payload;
  bool PayloadNil = true;  // Go distinguishes a nil slice (null) from an empty one ("")
  std::string String() const;  // message.go:51-62
};

Message NewConnect();                                                                   // message.go:25-27
Message NewData(int64_t connID, int64_t seqNum, int64_t size, const std::string& payload);  // message.go:31-39
Message NewAck(int64_t connID, int64_t seqNum);                                          // message.go:43-49

std::string Marshal(const Message& m);
// encoding/json.Unmarshal (gojson.hpp: Go 1.4's rules): true when Go's error
// would be nil; on a type error (e.g. a Payload that is not padded base64)
// *out holds the partial decode, on a syntax error it is untouched.  The LSP
// endpoints drop every datagram that is not error-free (lsp.cpp).
bool Unmarshal(const std::string& json, Message* out);
int UnmarshalStatus(const std::string& json, Message* out);  // gojson::Status

std::string Base64Encode(const std::vector<uint8_t>& b);
bool Base64Decode(const std::string& s, std::vector<uint8_t>* out);

}  // namespace lsp
