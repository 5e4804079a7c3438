// xml.hpp -- minimal, dependency-free XML reader for URDF/SRDF ingestion.
// Supports elements, attributes (single/double quoted), text, comments,
// processing instructions, <!DOCTYPE>, CDATA and the five predefined entities.
#pragma once

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mpgh {

struct XmlNode {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<XmlNode>> children;
  std::string text;

  const std::string* attr(const std::string& k) const {
    for (auto& a : attrs)
      if (a.first == k) return &a.second;
    return nullptr;
  }
  std::string attr_or(const std::string& k, const std::string& d) const {
    auto p = attr(k);
    return p ? *p : d;
  }
  const XmlNode* child(const std::string& t) const {
    for (auto& c : children)
      if (c->tag == t) return c.get();
    return nullptr;
  }
  std::vector<const XmlNode*> children_named(const std::string& t) const {
    std::vector<const XmlNode*> out;
    for (auto& c : children)
      if (c->tag == t) out.push_back(c.get());
    return out;
  }
};

class XmlParser {
 public:
  explicit XmlParser(const std::string& s) : s_(s) {}

  std::unique_ptr<XmlNode> parse() {
    skip_misc();
    if (pos_ >= s_.size() || s_[pos_] != '<') fail("expected root element");
    auto root = element();
    skip_misc();
    return root;
  }

 private:
  const std::string& s_;
  size_t pos_ = 0;

  [[noreturn]] void fail(const std::string& m) {
    throw std::invalid_argument("XML parse error at offset " + std::to_string(pos_) + ": " + m);
  }
  bool starts(const char* p) const { return s_.compare(pos_, std::char_traits<char>::length(p), p) == 0; }
  void ws() {
    while (pos_ < s_.size() && (s_[pos_] == ' ' || s_[pos_] == '\t' || s_[pos_] == '\n' || s_[pos_] == '\r')) ++pos_;
  }
  void skip_until(const char* end) {
    size_t e = s_.find(end, pos_);
    if (e == std::string::npos) fail(std::string("unterminated construct, expected ") + end);
    pos_ = e + std::char_traits<char>::length(end);
  }
  void skip_misc() {
    for (;;) {
      ws();
      if (starts("<?")) skip_until("?>");
      else if (starts("<!--")) skip_until("-->");
      else if (starts("<!DOCTYPE")) skip_until(">");
      else break;
    }
  }
  static std::string decode(const std::string& in) {
    std::string out;
    out.reserve(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
      if (in[i] == '&') {
        size_t e = in.find(';', i);
        if (e != std::string::npos) {
          std::string ent = in.substr(i + 1, e - i - 1);
          if (ent == "lt") { out += '<'; i = e; continue; }
          if (ent == "gt") { out += '>'; i = e; continue; }
          if (ent == "amp") { out += '&'; i = e; continue; }
          if (ent == "quot") { out += '"'; i = e; continue; }
          if (ent == "apos") { out += '\''; i = e; continue; }
        }
      }
      out += in[i];
    }
    return out;
  }
  std::string name() {
    size_t b = pos_;
    while (pos_ < s_.size() && !strchr(" \t\r\n/>=", s_[pos_])) ++pos_;
    if (b == pos_) fail("expected a name");
    return s_.substr(b, pos_ - b);
  }
  std::unique_ptr<XmlNode> element() {
    ++pos_;  // '<'
    auto n = std::make_unique<XmlNode>();
    n->tag = name();
    for (;;) {
      ws();
      if (pos_ >= s_.size()) fail("unexpected end in tag");
      if (starts("/>")) {
        pos_ += 2;
        return n;
      }
      if (s_[pos_] == '>') {
        ++pos_;
        break;
      }
      std::string k = name();
      ws();
      if (s_[pos_] != '=') fail("expected '=' after attribute " + k);
      ++pos_;
      ws();
      char q = s_[pos_];
      if (q != '"' && q != '\'') fail("expected quoted attribute value");
      size_t e = s_.find(q, pos_ + 1);
      if (e == std::string::npos) fail("unterminated attribute value");
      n->attrs.emplace_back(k, decode(s_.substr(pos_ + 1, e - pos_ - 1)));
      pos_ = e + 1;
    }
    for (;;) {
      if (pos_ >= s_.size()) fail("unterminated element <" + n->tag + ">");
      if (starts("<!--")) {
        skip_until("-->");
      } else if (starts("<![CDATA[")) {
        size_t b = pos_ + 9;
        skip_until("]]>");
        n->text += s_.substr(b, pos_ - 3 - b);
      } else if (starts("<?")) {
        skip_until("?>");
      } else if (starts("</")) {
        pos_ += 2;
        std::string t = name();
        if (t != n->tag) fail("mismatched </" + t + "> for <" + n->tag + ">");
        ws();
        if (s_[pos_] != '>') fail("expected '>'");
        ++pos_;
        return n;
      } else if (s_[pos_] == '<') {
        n->children.push_back(element());
      } else {
        size_t e = s_.find('<', pos_);
        if (e == std::string::npos) fail("unterminated text");
        n->text += decode(s_.substr(pos_, e - pos_));
        pos_ = e;
      }
    }
  }
};

}  // namespace mpgh
