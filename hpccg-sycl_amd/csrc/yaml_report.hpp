// yaml_report.hpp -- writer for the Mantevo-style report test_HPCCG prints.
//
// Output format is the reference's (YAML_Doc.cpp:32-72, YAML_Element.cpp:
// 87-99): "key: value" lines, two spaces of indent per level, numbers through
// a default-formatted ostream (6 significant digits), a header with the
// mini-app name and version, and a copy written to
// ./<name>-<version>_YYYY_MM_DD__HH_MM_SS.yaml.
#pragma once
#include <ctime>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

namespace hpccg {

class Report {
public:
    struct Node {
        std::string key, value;
        std::vector<std::unique_ptr<Node>> kids;

        template <class T>
        Node* add(const std::string& k, const T& v)
        {
            std::ostringstream os;
            os << v;
            return put(k, os.str());
        }
        Node* add(const std::string& k, const char* v) { return put(k, v); }
        Node* add(const std::string& k, const std::string& v) { return put(k, v); }
        Node* get(const std::string& k)
        {
            for (auto& c : kids)
                if (c->key == k) return c.get();
            return nullptr;
        }
        void emit(std::string& out, const std::string& indent) const
        {
            out += indent + key + ": " + value + "\n";
            for (auto& c : kids) c->emit(out, indent + "  ");
        }

    private:
        Node* put(const std::string& k, const std::string& v)
        {
            value.clear();  // a node with children carries no value
            kids.emplace_back(new Node{k, v, {}});
            return kids.back().get();
        }
    };

    Report(std::string name, std::string version) : name_(std::move(name)), version_(std::move(version)) {}

    template <class T>
    Node* add(const std::string& k, const T& v) { return root_.add(k, v); }
    Node* get(const std::string& k) { return root_.get(k); }

    // Renders the document and writes the time-stamped copy; returns the text.
    std::string render(bool write_file = true) const
    {
        std::string out = "Mini-Application Name: " + name_ + "\n";
        out += "Mini-Application Version: " + version_ + "\n";
        for (auto& c : root_.kids) c->emit(out, "");
        if (write_file) {
            std::time_t now = std::time(nullptr);
            std::tm* t = std::localtime(&now);
            char stamp[96];
            std::snprintf(stamp, sizeof stamp, "%04d_%02d_%02d__%02d_%02d_%02d", t->tm_year + 1900,
                          t->tm_mon + 1, t->tm_mday, t->tm_hour, t->tm_min, t->tm_sec);
            std::ofstream f("./" + name_ + "-" + version_ + "_" + stamp + ".yaml");
            f << out;
        }
        return out;
    }

private:
    std::string name_, version_;
    Node root_;
};

}  // namespace hpccg
