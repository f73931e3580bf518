// test_mirror.cpp — the reference's own unit tests, restated against the C++
// mirror types (include/onc_rpc.hpp) running on the GPU codec.
//
// Each test names the reference test it follows. Byte vectors are read from
// tests/golden/vectors.json (fixtures extracted from the reference's tests,
// see tests/golden/make_golden.py). Run by tests/test_cpp_mirror.py (-m gpu).
//
// Usage: test_mirror <path to vectors.json>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/onc_rpc.hpp"

using namespace onc_rpc;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                                  \
    do {                                                                             \
        if (!(cond)) {                                                               \
            std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            throw std::runtime_error("check failed");                                \
        }                                                                            \
    } while (0)

// ---- minimal fixture reader: the entry whose "name" is `name` ------------------
static std::string g_json;

static std::string entry(const std::string& name) {
    const std::string key = "\"name\": \"" + name + "\"";
    const size_t a = g_json.find(key);
    if (a == std::string::npos) throw std::runtime_error("no fixture " + name);
    size_t b = g_json.find("\"name\": \"", a + key.size());
    return g_json.substr(a, b == std::string::npos ? std::string::npos : b - a);
}

static std::string field_str(const std::string& e, const std::string& f) {
    const std::string key = "\"" + f + "\": \"";
    const size_t a = e.find(key);
    if (a == std::string::npos) throw std::runtime_error("no field " + f);
    const size_t s = a + key.size();
    return e.substr(s, e.find('"', s) - s);
}

static long field_int(const std::string& e, const std::string& f) {
    const std::string key = "\"" + f + "\": ";
    const size_t a = e.find(key);
    if (a == std::string::npos) throw std::runtime_error("no field " + f);
    return std::stol(e.substr(a + key.size()));
}

static std::vector<uint8_t> unhex(const std::string& h) {
    std::vector<uint8_t> v(h.size() / 2);
    for (size_t i = 0; i < v.size(); ++i) v[i] = uint8_t(std::stoi(h.substr(2 * i, 2), nullptr, 16));
    return v;
}

static std::vector<uint8_t> fixture(const std::string& name) { return unhex(field_str(entry(name), "hex")); }

static std::vector<uint32_t> gids16() {
    return {501, 12, 20, 61, 79, 80, 81, 98, 701, 33, 100, 204, 250, 395, 398, 399};
}

// ---- tests ----------------------------------------------------------------------

// rpc_message.rs:446-580 test_rpcmessage_auth_unix (+ Bytes variant :582-719)
static void test_rpcmessage_auth_unix(Codec& c) {
    const std::vector<uint8_t> raw = fixture("call_auth_unix_16gids_288B");
    for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
        const RpcMessage msg = RpcMessage::try_from(c, Bytes(raw), mode);
        CHECK(msg.xid() == 643743997);
        CHECK(msg.serialised_len(c) == 288);
        const CallBody* body = msg.call_body();
        CHECK(body != nullptr && msg.reply_body() == nullptr);
        CHECK(body->rpc_version() == 2);
        CHECK(body->program() == 100003);
        CHECK(body->program_version() == 4);
        CHECK(body->procedure() == 1);
        CHECK(body->auth_credentials().kind() == AuthFlavor::Kind::AuthUnix);
        const AuthUnixParams& p = body->auth_credentials().unix_params();
        CHECK(p.stamp() == 0);
        CHECK(p.machine_name().len == 0);
        CHECK(p.uid() == 501);
        CHECK(p.gid() == 20);
        CHECK(p.gids().has_value() && *p.gids() == gids16());
        CHECK(body->auth_verifier() == AuthFlavor::none());
        CHECK(body->payload().len == 288 - 4 - 4 - 4 - 16 - 92 - 8);
        // borrowed, zero-copy: the payload view points into `raw`
        CHECK(body->payload().ptr == raw.data() + (288 - body->payload().len));
        // re-serialise -> identical bytes
        CHECK(msg.serialise(c) == raw);
    }
}

// rpc_message.rs:790-796 (call with one gid; also benches/bench.rs:55-60)
static void test_rpcmessage_auth_unix_1gid(Codec& c) {
    const std::vector<uint8_t> raw = fixture("call_auth_unix_1gid_156B");
    const RpcMessage msg = RpcMessage::try_from(c, Bytes(raw));
    CHECK(msg.xid() == 643744006);
    CHECK(msg.call_body()->auth_credentials().unix_params().gids() == std::vector<uint32_t>{0});
    CHECK(msg.serialise(c) == raw);
}

// rpc_message.rs:849-853 test_rpcmessage_reply (accepted success)
static void test_rpcmessage_reply(Codec& c) {
    const std::vector<uint8_t> raw = fixture("reply_accepted_success_76B");
    for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
        const RpcMessage msg = RpcMessage::try_from(c, Bytes(raw), mode);
        CHECK(msg.xid() == 643743997);
        const ReplyBody* r = msg.reply_body();
        CHECK(r != nullptr && r->is_accepted());
        CHECK(r->accepted()->auth_verifier() == AuthFlavor::none());
        CHECK(r->accepted()->status().kind() == AcceptedStatus::Kind::Success);
        CHECK(r->accepted()->status().payload().len == 48);
        CHECK(msg.serialised_len(c) == 76);
        CHECK(msg.serialise(c) == raw);
    }
}

// rpc_message.rs:937-940 (fuzz-found reply with trailing bytes) and the
// unwrap_header error vectors (:388-427): exact Error variant and payload.
static void test_error_vectors(Codec& c) {
    for (const char* name : {"fuzz_reply_too_long_for_type_39B", "unwrap_header_incomplete_header",
                             "unwrap_header_incomplete_message", "unwrap_header_fragmented"}) {
        const std::string e = entry(name);
        const std::vector<uint8_t> raw = unhex(field_str(e, "hex"));
        const long want = field_int(e, "status");
        for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
            bool threw = false;
            try {
                (void)RpcMessage::try_from(c, Bytes(raw), mode);
            } catch (const Error& err) {
                threw = true;
                CHECK(err.code() == want);
                if (want == ONC_ERR_INCOMPLETE_MESSAGE) {
                    CHECK(err.buffer_len() == uint32_t(field_int(e, "aux0")));
                    CHECK(err.expected() == uint32_t(field_int(e, "aux1")));
                }
            }
            CHECK(threw);
        }
    }
}

// rpc_message.rs:171-190 doc example: CallBody with AuthNone x2, no payload.
static void test_doc_example(Codec& c) {
    const std::vector<uint8_t> want = fixture("doc_example_call_none_none_empty");
    const RpcMessage msg(4242, MessageType::call(CallBody(100000, 42, 13, AuthFlavor::none(), AuthFlavor::none(),
                                                          Bytes())));
    CHECK(msg.serialised_len(c) == want.size());
    CHECK(msg.serialise(c) == want);
    // serialise_into appends (a Cursor positioned at the end of a Vec)
    std::vector<uint8_t> buf = {0xAA};
    msg.serialise_into(c, buf);
    CHECK(buf.size() == want.size() + 1 && buf[0] == 0xAA);
    CHECK(std::vector<uint8_t>(buf.begin() + 1, buf.end()) == want);
}

// benches/bench.rs:86-101: the reference benchmark's round trip (configs[0]).
static void test_bench_message_round_trip(Codec& c) {
    std::vector<uint8_t> payload(64);
    for (size_t i = 0; i < payload.size(); ++i) payload[i] = uint8_t(i * 7 + 3);
    const RpcMessage msg(4242, MessageType::call(CallBody(
                                   100000, 42, 13, AuthFlavor::unix(AuthUnixParams(0, Bytes(), 501, 20, gids16())),
                                   AuthFlavor::none(), Bytes(payload))));
    const std::vector<uint8_t> wire = msg.serialise(c);
    CHECK(wire.size() == 192);   // W = 192
    const RpcMessage back = RpcMessage::try_from(c, Bytes(wire));
    CHECK(back.xid() == msg.xid());
    CHECK(back.call_body()->auth_credentials() == msg.call_body()->auth_credentials());
    CHECK(back.call_body()->payload() == Bytes(payload));
    CHECK(back == msg);
}

// What the single-message calls cost (onc_rpc.hpp): RpcMessage::serialise /
// try_from on a Codec are whole GPU round trips (host arenas -> device,
// kernels, device -> host, a stream sync each), meant for tests and tiny
// batches; BatchEncoder / BatchDecoder amortise that over a batch. The
// configs[0] message (benches/bench.rs:86-101): 200 single-message round
// trips against one 200-message batch round trip, printed as TIMING lines.
static void test_single_message_cost(Codec& c) {
    std::vector<uint8_t> payload(64);
    for (size_t i = 0; i < payload.size(); ++i) payload[i] = uint8_t(i * 5 + 1);
    const RpcMessage msg(7, MessageType::call(CallBody(100000, 42, 13,
                                                       AuthFlavor::unix(AuthUnixParams(0, Bytes(), 501, 20, gids16())),
                                                       AuthFlavor::none(), Bytes(payload))));
    constexpr int kN = 200;
    (void)RpcMessage::try_from(c, Bytes(msg.serialise(c)));     // warm-up
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < kN; ++i) {
        const std::vector<uint8_t> w = msg.serialise(c);
        CHECK(RpcMessage::try_from(c, Bytes(w)) == msg);
    }
    const auto t1 = std::chrono::steady_clock::now();
    BatchEncoder enc;
    for (int i = 0; i < kN; ++i) enc.push(msg);
    std::vector<uint8_t> wire;
    std::vector<uint64_t> off;
    (void)enc.serialise_into(c, wire, &off);                     // warm-up
    const auto t2 = std::chrono::steady_clock::now();
    wire.clear();
    const std::vector<int32_t> st = enc.serialise_into(c, wire, &off);
    std::vector<uint32_t> rec_len(kN);
    for (int i = 0; i < kN; ++i) rec_len[i] = uint32_t(off[i + 1] - off[i]);
    BatchDecoder dec;
    const std::vector<Decoded> out = dec.try_from(c, wire.data(), wire.size(), rec_len);
    const auto t3 = std::chrono::steady_clock::now();
    for (int i = 0; i < kN; ++i) CHECK(st[i] == ONC_OK && out[i].ok() && *out[i].message == msg);
    const double single = std::chrono::duration<double, std::micro>(t1 - t0).count() / kN;
    const double batch = std::chrono::duration<double, std::micro>(t3 - t2).count();
    std::printf("TIMING single_message_round_trip_us=%.1f batch_%d_round_trip_us=%.1f per_message_in_batch_us=%.2f\n",
                single, kN, batch, batch / kN);
}

// Panic parity: flavor.rs:110 (assoc > 200), unix_params.rs:149 (name > 255),
// unix_params.rs:47 (> 16 gids) -> std::logic_error.
static void test_panics(Codec& c) {
    bool threw = false;
    try {
        AuthUnixParams(0, Bytes(), 0, 0, std::vector<uint32_t>(17, 1));
    } catch (const std::logic_error&) {
        threw = true;
    }
    CHECK(threw);
    std::vector<uint8_t> big(256, 'x');
    threw = false;
    try {
        AuthUnixParams(0, Bytes(big), 0, 0, {});
    } catch (const std::logic_error&) {
        threw = true;
    }
    CHECK(threw);
    // 201 bytes of AuthNone data: the reference panics in serialise_into
    std::vector<uint8_t> body(201, 1);
    const RpcMessage m(1, MessageType::call(CallBody(1, 1, 1, AuthFlavor::none(Bytes(body)), AuthFlavor::none(),
                                                     Bytes())));
    threw = false;
    try {
        (void)m.serialise(c);
    } catch (const std::logic_error&) {
        threw = true;
    }
    CHECK(threw);
    // exactly 200 is fine (flavor.rs:110 is <=)
    std::vector<uint8_t> ok(200, 2);
    const RpcMessage m2(1, MessageType::call(CallBody(1, 1, 1, AuthFlavor::short_(Bytes(ok)), AuthFlavor::none(),
                                                      Bytes())));
    CHECK(m2.serialise(c).size() == 4 + 4 + 4 + 16 + 8 + 200 + 8);
}

// rpc_message.rs:343-367 expected_message_len
static void test_expected_message_len(Codec&) {
    const std::vector<uint8_t> raw = fixture("call_auth_unix_16gids_288B");
    CHECK(expected_message_len(Bytes(raw)) == 288);
    bool threw = false;
    try {
        expected_message_len(Bytes(raw.data(), 3));
    } catch (const Error& e) {
        threw = e.code() == ONC_ERR_INCOMPLETE_HEADER;
    }
    CHECK(threw);
    const uint8_t frag[4] = {0, 0, 0, 8};
    threw = false;
    try {
        expected_message_len(Bytes(frag, 4));
    } catch (const Error& e) {
        threw = e.code() == ONC_ERR_FRAGMENTED;
    }
    CHECK(threw);
}

// Property test (rpc_message.rs:1134-1153 proptest invariants) over the batch
// classes: every variant, serialise -> try_from -> equal, lengths agree.
static void test_batch_round_trip(Codec& c) {
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return uint32_t((z ^ (z >> 31)) >> 7);
    };
    std::vector<std::vector<uint8_t>> store;
    auto bytes = [&](size_t n) {
        store.emplace_back(n);
        for (auto& b : store.back()) b = uint8_t(rnd());
        return Bytes(store.back());
    };
    store.reserve(20000);
    auto auth = [&]() -> AuthFlavor {
        switch (rnd() % 5) {
            case 0: return AuthFlavor::none();
            case 1: return AuthFlavor::none(bytes(1 + rnd() % 200));
            case 2: {
                std::vector<uint32_t> g(rnd() % 17);
                for (auto& x : g) x = rnd();
                return AuthFlavor::unix(AuthUnixParams(rnd(), bytes(rnd() % 40), rnd(), rnd(), g));
            }
            case 3: return AuthFlavor::short_(bytes(rnd() % 200));
            default: return AuthFlavor::unknown(3 + rnd() % 1000, bytes(rnd() % 200));
        }
    };
    std::vector<RpcMessage> msgs;
    BatchEncoder enc;
    for (int i = 0; i < 3000; ++i) {
        const uint32_t k = rnd() % 6;
        if (k < 3) {
            msgs.emplace_back(rnd(), MessageType::call(CallBody(rnd(), rnd(), rnd(), auth(), auth(), bytes(rnd() % 700))));
        } else if (k == 3) {
            AcceptedStatus st = AcceptedStatus::success(bytes(rnd() % 700));
            const uint32_t w = rnd() % 6;
            if (w == 2) st = AcceptedStatus::program_mismatch(rnd(), rnd());
            else if (w) st = AcceptedStatus::of(AcceptedStatus::Kind(w));
            msgs.emplace_back(rnd(), MessageType::reply(ReplyBody::accepted(AcceptedReply(auth(), st))));
        } else if (k == 4) {
            msgs.emplace_back(rnd(), MessageType::reply(ReplyBody::denied(
                                         RejectedReply::rpc_version_mismatch(rnd(), rnd()))));
        } else {
            msgs.emplace_back(rnd(), MessageType::reply(ReplyBody::denied(
                                         RejectedReply::auth_error(AuthError(rnd() % 8)))));
        }
        enc.push(msgs.back());
    }
    std::vector<uint8_t> wire;
    std::vector<uint64_t> off;
    const std::vector<int32_t> st = enc.serialise_into(c, wire, &off);
    const std::vector<uint32_t> lens = enc.serialised_lens(c);
    std::vector<uint32_t> rec_len(msgs.size());
    for (size_t i = 0; i < msgs.size(); ++i) {
        CHECK(st[i] == ONC_OK);
        rec_len[i] = uint32_t(off[i + 1] - off[i]);
        CHECK(rec_len[i] == lens[i]);
    }
    BatchDecoder dec;
    for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
        const std::vector<Decoded> out = dec.try_from(c, wire.data(), wire.size(), rec_len, mode);
        for (size_t i = 0; i < msgs.size(); ++i) {
            CHECK(out[i].ok());
            CHECK(*out[i].message == msgs[i]);
        }
    }
    // the same send buffer registered (onc_host_register) and decoded where it lies
    const HostRegistration reg(c, wire.data(), wire.size());
    for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
        const std::vector<Decoded> out = dec.try_from(c, reg, rec_len, mode);
        CHECK(out.size() == msgs.size());
        for (size_t i = 0; i < msgs.size(); ++i) {
            CHECK(out[i].ok());
            CHECK(*out[i].message == msgs[i]);
        }
    }
    size_t consumed = 0;
    std::optional<Error> stop;
    const std::vector<Decoded> framed = dec.try_from_stream(c, reg, DecodeMode::Slice, &consumed, &stop);
    CHECK(framed.size() == msgs.size() && consumed == wire.size() && !stop.has_value());
    for (size_t i = 0; i < msgs.size(); ++i) CHECK(framed[i].ok() && *framed[i].message == msgs[i]);
}

// The caller's loop over a socket buffer (expected_message_len + one-message
// slices), done on the device: BatchDecoder::try_from_stream.
static void test_stream_framing(Codec& c) {
    const std::vector<uint8_t> a = fixture("call_auth_unix_16gids_288B");
    const std::vector<uint8_t> b = fixture("reply_accepted_success_76B");
    std::vector<uint8_t> stream;
    for (int i = 0; i < 500; ++i) {
        const std::vector<uint8_t>& r = (i % 3) ? a : b;
        stream.insert(stream.end(), r.begin(), r.end());
    }
    BatchDecoder dec;
    size_t consumed = 0;
    std::optional<Error> stop;
    std::vector<Decoded> out = dec.try_from_stream(c, stream.data(), stream.size(), DecodeMode::Slice, &consumed, &stop);
    CHECK(out.size() == 500 && consumed == stream.size() && !stop.has_value());
    for (int i = 0; i < 500; ++i) {
        CHECK(out[i].ok());
        CHECK(out[i].message->xid() == ((i % 3) ? 643743997u : 643743997u));
        CHECK((out[i].message->call_body() != nullptr) == bool(i % 3));
    }
    // a partial trailing record: "read more" (IncompleteMessage), 499 framed
    out = dec.try_from_stream(c, stream.data(), stream.size() - 10, DecodeMode::Bytes, &consumed, &stop);
    CHECK(out.size() == 499 && consumed == stream.size() - a.size());
    CHECK(stop.has_value() && stop->code() == ONC_ERR_INCOMPLETE_MESSAGE);
    CHECK(stop->buffer_len() == a.size() - 10 && stop->expected() == a.size());
}

// A 16 MiB socket buffer framed and decoded by a fresh codec: the stage holds
// the wire and the offsets while framing, and the decode outputs only for the
// records framed (it grows keeping the staged wire; sized for every possible
// 4-byte record the outputs alone would be ~1.1 GB of pinned memory).
static void test_stream_stage_size(Codec&) {
    Codec c(0);
    const std::vector<uint8_t> a = fixture("call_auth_unix_16gids_288B");
    std::vector<uint8_t> stream;
    while (stream.size() + a.size() <= (size_t(16) << 20)) stream.insert(stream.end(), a.begin(), a.end());
    const size_t n = stream.size() / a.size();
    BatchDecoder dec;
    size_t consumed = 0;
    std::optional<Error> stop;
    const std::vector<Decoded> out = dec.try_from_stream(c, stream.data(), stream.size(), DecodeMode::Slice,
                                                         &consumed, &stop);
    CHECK(out.size() == n && consumed == stream.size() && !stop.has_value());
    for (size_t i = 0; i < n; i += 997) CHECK(out[i].ok() && out[i].message->xid() == 643743997u);
    CHECK(out[n - 1].ok());
    std::printf("  stream of %zu bytes (%zu records): stage %zu MiB\n", stream.size(), n, c.stage_capacity() >> 20);
    CHECK(c.stage_capacity() <= (size_t(128) << 20));
}

// ---- body-level types (onc_decode_body / onc_encode_body) -----------------------

// flavor.rs:232-266 test_auth_unix_unaligned_machinename, :268-320 test_auth_unix
static void test_auth_unix_flavors(Codec& c) {
    for (const char* name : {"auth_unix_unaligned_machine_name", "auth_unix_16gids"}) {
        const std::vector<uint8_t> raw = fixture(name);
        for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
            const AuthFlavor f = AuthFlavor::try_from(c, Bytes(raw), mode);
            CHECK(f.serialised_len(c) == raw.size());
            CHECK(f.id() == ONC_AUTH_UNIX);
            CHECK(f.kind() == AuthFlavor::Kind::AuthUnix);
            const bool unaligned = raw.size() == 44;
            CHECK(f.associated_data_len() == (unaligned ? 27u : 92u - 4 - 4 - 4 - 4));
            CHECK(f.unix_params().uid() == (unaligned ? 0u : 501u));
            if (unaligned) CHECK(f.unix_params().machine_name_str() == "LAPTOP-1QQBPDGM");
            else CHECK(f.unix_params().gids() == gids16());
            std::vector<uint8_t> out;
            f.serialise_into(c, out);
            CHECK(out == raw);
        }
    }
}

// flavor.rs:322-344 test_auth_none, :346-368 test_auth_short, :370-393 test_auth_unknown
static void test_auth_opaque_flavors(Codec& c) {
    const std::pair<const char*, AuthFlavor::Kind> cases[] = {{"auth_none_with_data", AuthFlavor::Kind::AuthNone},
                                                              {"auth_short", AuthFlavor::Kind::AuthShort},
                                                              {"auth_unknown_255", AuthFlavor::Kind::Unknown}};
    for (const auto& cs : cases) {
        const std::vector<uint8_t> raw = fixture(cs.first);
        for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
            const AuthFlavor f = AuthFlavor::try_from(c, Bytes(raw), mode);
            CHECK(f.kind() == cs.second);
            CHECK(f.serialised_len(c) == 92);
            CHECK(f.id() == (cs.second == AuthFlavor::Kind::AuthNone    ? 0u
                             : cs.second == AuthFlavor::Kind::AuthShort ? 2u
                                                                        : 255u));
            CHECK(f.associated_data_len() == 92 - 4 - 4);
            CHECK(f.data().has_value() && f.data()->len == f.associated_data_len());
            CHECK(f.data()->ptr == raw.data() + 8);     // borrowed
            std::vector<uint8_t> out;
            f.serialise_into(c, out);
            CHECK(out == raw);
        }
    }
}

// unix_params.rs:287-344 test_serialise_deserialise / :381-435 (Bytes),
// :346-379 test_empty / :437-471 (Bytes)
static void test_auth_unix_params(Codec& c) {
    const std::vector<uint8_t> raw16 = fixture("unix_params_16gids_84B");
    const std::vector<uint8_t> raw1 = fixture("unix_params_1gid_24B");
    const AuthUnixParams want16(0, Bytes(), 501, 20, gids16());
    const AuthUnixParams want1(0, Bytes(), 0, 0, {0});
    std::vector<uint8_t> out;
    want16.serialise_into(c, out);
    CHECK(out == raw16);
    CHECK(want16.serialised_len(c) == 84);
    out.clear();
    want1.serialise_into(c, out);
    CHECK(out == raw1);
    CHECK(AuthUnixParams::from_cursor(c, Bytes(raw16), 84) == want16);
    CHECK(AuthUnixParams::try_from(c, Bytes(raw16)) == want16);
    CHECK(AuthUnixParams::from_cursor(c, Bytes(raw1), 24) == want1);
    CHECK(AuthUnixParams::try_from(c, Bytes(raw1)) == want1);
    // from_cursor checks the consumed length (unix_params.rs:117-119)
    bool threw = false;
    try {
        (void)AuthUnixParams::from_cursor(c, Bytes(raw1), 28);
    } catch (const Error& e) {
        threw = e.code() == ONC_ERR_INVALID_AUTH_DATA;
    }
    CHECK(threw);
}

// The call and reply bodies of the whole-message vectors, each as its own
// type: CallBody (call_body.rs:168-210), ReplyBody (reply_body.rs:76-98),
// AcceptedReply / AcceptedStatus (accepted_reply.rs:79-105, :234-265).
static void test_body_types(Codec& c) {
    const std::vector<uint8_t> call = fixture("call_auth_unix_16gids_288B");
    const std::vector<uint8_t> reply = fixture("reply_accepted_success_76B");
    for (DecodeMode mode : {DecodeMode::Slice, DecodeMode::Bytes}) {
        const RpcMessage m = RpcMessage::try_from(c, Bytes(call), mode);
        const Bytes cb(call.data() + 12, call.size() - 12);
        const CallBody b = CallBody::try_from(c, cb, mode);
        CHECK(b == *m.call_body());
        CHECK(b.serialised_len(c) == cb.len);
        std::vector<uint8_t> out;
        b.serialise_into(c, out);
        CHECK(Bytes(out) == cb);
        const MessageType t = MessageType::try_from(c, Bytes(call.data() + 8, call.size() - 8), mode);
        CHECK(t == m.message());
        CHECK(t.serialised_len(c) == call.size() - 8);

        const RpcMessage r = RpcMessage::try_from(c, Bytes(reply), mode);
        const Bytes rb(reply.data() + 12, reply.size() - 12);
        const ReplyBody rbody = ReplyBody::try_from(c, rb, mode);
        CHECK(rbody == *r.reply_body());
        out.clear();
        rbody.serialise_into(c, out);
        CHECK(Bytes(out) == rb);
        const AcceptedReply ar = AcceptedReply::try_from(c, Bytes(rb.ptr + 4, rb.len - 4), mode);
        CHECK(ar == *r.reply_body()->accepted());
        CHECK(ar.serialised_len(c) == rb.len - 4);
        const AcceptedStatus as = AcceptedStatus::try_from(c, Bytes(rb.ptr + 12, rb.len - 12), mode);
        CHECK(as.kind() == AcceptedStatus::Kind::Success && as.payload().len == 48);
        out.clear();
        as.serialise_into(c, out);
        CHECK(Bytes(out) == Bytes(rb.ptr + 12, rb.len - 12));
    }
    // rejected replies and auth errors, built then parsed back
    for (const RejectedReply& j : {RejectedReply::rpc_version_mismatch(2, 5), RejectedReply::auth_error(AuthError::TooWeak)}) {
        std::vector<uint8_t> out;
        j.serialise_into(c, out);
        CHECK(out.size() == j.serialised_len(c));
        CHECK(RejectedReply::try_from(c, Bytes(out)) == j);
        CHECK(RejectedReply::try_from(c, Bytes(out), DecodeMode::Bytes) == j);
    }
    std::vector<uint8_t> e;
    serialise_into(c, AuthError::InvalidResponseVerifier, e);
    CHECK(e == (std::vector<uint8_t>{0, 0, 0, 6}));
    CHECK(auth_error_try_from(c, Bytes(e)) == AuthError::InvalidResponseVerifier);
    const std::vector<uint8_t> bad = {0, 0, 0, 8};
    bool threw = false;
    try {
        (void)auth_error_try_from(c, Bytes(bad), DecodeMode::Bytes);
    } catch (const Error& x) {
        threw = x.code() == ONC_ERR_INVALID_AUTH_ERROR && x.value() == 8;
    }
    CHECK(threw);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s vectors.json\n", argv[0]);
        return 2;
    }
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    g_json = ss.str();
    if (g_json.empty()) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    Codec codec(0);
    const std::vector<std::pair<const char*, std::function<void(Codec&)>>> tests = {
        {"test_rpcmessage_auth_unix", test_rpcmessage_auth_unix},
        {"test_rpcmessage_auth_unix_1gid", test_rpcmessage_auth_unix_1gid},
        {"test_rpcmessage_reply", test_rpcmessage_reply},
        {"test_error_vectors", test_error_vectors},
        {"test_doc_example", test_doc_example},
        {"test_bench_message_round_trip", test_bench_message_round_trip},
        {"test_panics", test_panics},
        {"test_expected_message_len", test_expected_message_len},
        {"test_batch_round_trip", test_batch_round_trip},
        {"test_stream_framing", test_stream_framing},
        {"test_stream_stage_size", test_stream_stage_size},
        {"test_auth_unix_flavors", test_auth_unix_flavors},
        {"test_auth_opaque_flavors", test_auth_opaque_flavors},
        {"test_auth_unix_params", test_auth_unix_params},
        {"test_body_types", test_body_types},
        {"test_single_message_cost", test_single_message_cost},
    };
    for (const auto& t : tests) {
        try {
            t.second(codec);
            ++g_pass;
            std::printf("PASS %s\n", t.first);
        } catch (const std::exception& e) {
            ++g_fail;
            std::printf("FAIL %s: %s\n", t.first, e.what());
        }
    }
    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
