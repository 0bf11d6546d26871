// config.cpp — system / workspace configuration files.
//
// The reference hardcodes its configuration in demos/main.cu:19-46, ships an
// empty systems/car.yaml and links yaml-cpp without calling it (CMakeLists.txt:10,
// 47); configurations/{init,goal,numR1,R2}/*.csv are never read.  Here one parser,
// behind the C ABI (sbmp_load_system_config), serves the C++ demo, the header-only
// facade, the Python mirror and bench.py, so a configuration (c1-c5, the demo) is
// chosen without recompiling.  yaml-cpp is not available, so the accepted format is
// the flat subset the files use:
//   key: value        # comment
// with a value a number, true / false, a word (car, point, reference, fill), a
// [x, y, ...] list, or a path (relative to the file's directory).  A numeric key
// may name a file holding the number (N: ../configurations/numR1/numR1.csv), and
// initial / goal a CSV file of 7 values (../configurations/init/init.csv).  Unknown
// keys are errors (a misspelt key would otherwise fall back to the demo silently).
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "kgmt_planner.h"
#include "sbmp/sbmp.h"

namespace sbmp {

static std::string trim(const std::string& s) {
    const size_t a = s.find_first_not_of(" \t\r");
    if (a == std::string::npos) return "";
    const size_t b = s.find_last_not_of(" \t\r");
    return s.substr(a, b - a + 1);
}

static std::string resolve(const std::string& base, std::string p) {
    if (p.size() >= 2 && (p.front() == '"' || p.front() == '\'') && p.back() == p.front()) p = p.substr(1, p.size() - 2);
    if (p.empty() || p[0] == '/') return p;
    return base.empty() ? p : base + "/" + p;
}

// Numbers separated by commas and/or whitespace (readObstaclesFromCSV's tolerance,
// helper.cu:11-34).
static std::vector<double> numbers_of(const std::string& text) {
    std::string t = text;
    for (char& c : t)
        if (c == ',' || c == '[' || c == ']') c = ' ';
    std::istringstream ss(t);
    std::vector<double> v;
    std::string tok;
    while (ss >> tok) {
        char* end = nullptr;
        errno = 0;
        const double x = std::strtod(tok.c_str(), &end);
        if (end == tok.c_str() || *end != '\0' || errno == ERANGE) return {};
        v.push_back(x);
    }
    return v;
}

static std::vector<double> numbers_from(const std::string& base, const std::string& key, const std::string& value) {
    std::vector<double> v = numbers_of(value);
    if (!v.empty()) return v;
    const std::string path = resolve(base, value);
    std::ifstream f(path);
    if (!f.is_open()) throw Error(SBMP_ERR_IO, key + ": '" + value + "' is neither numbers nor a readable file");
    std::stringstream buf;
    buf << f.rdbuf();
    v = numbers_of(buf.str());
    if (v.empty()) throw Error(SBMP_ERR_INVALID_ARGUMENT, key + ": no numbers in " + path);
    return v;
}

static double scalar(const std::string& base, const std::string& key, const std::string& value) {
    const std::vector<double> v = numbers_from(base, key, value);
    return v[0];
}

static int integer(const std::string& base, const std::string& key, const std::string& value) {
    const double x = scalar(base, key, value);
    if (x != std::floor(x) || std::fabs(x) > 2147483647.0)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, key + " must be an integer");
    return (int)x;
}

static int boolean(const std::string& key, const std::string& value) {
    if (value == "true" || value == "1") return 1;
    if (value == "false" || value == "0") return 0;
    throw Error(SBMP_ERR_INVALID_ARGUMENT, key + " must be true or false");
}

void load_system_config(const char* path, sbmp_system_config* out) {
    if (!path || !out) throw Error(SBMP_ERR_INVALID_ARGUMENT, "NULL argument");
    std::ifstream f(path);
    if (!f.is_open()) throw Error(SBMP_ERR_IO, std::string("cannot open ") + path);
    sbmp_system_config c;
    memset(&c, 0, sizeof(c));
    if (sbmp_kgmt_default_params(&c.params) != SBMP_OK) throw Error(SBMP_ERR_INVALID_ARGUMENT, "default params");
    const float demoInit[7] = {5, 5, 0, 0, 0, 0, 0}, demoGoal[7] = {2, 18, 0, 0, 0, 0, 0};   // main.cu:33-45
    memcpy(c.initial, demoInit, sizeof(demoInit));
    memcpy(c.goal, demoGoal, sizeof(demoGoal));
    const std::string p(path);
    const size_t slash = p.find_last_of('/');
    const std::string base = slash == std::string::npos ? "" : p.substr(0, slash);
    std::string line;
    int lineNo = 0;
    while (std::getline(f, line)) {
        ++lineNo;
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        line = trim(line);
        if (line.empty()) continue;
        const size_t colon = line.find(':');
        if (colon == std::string::npos)
            throw Error(SBMP_ERR_INVALID_ARGUMENT, p + ":" + std::to_string(lineNo) + ": expected key: value");
        const std::string key = trim(line.substr(0, colon)), value = trim(line.substr(colon + 1));
        sbmp_kgmt_params& q = c.params;
        if (key == "agent") {
            if (value == "car") q.agent = SBMP_AGENT_CAR;
            else if (value == "point") q.agent = SBMP_AGENT_POINT;
            else throw Error(SBMP_ERR_INVALID_ARGUMENT, "agent must be car or point");
        } else if (key == "width") q.width = (float)scalar(base, key, value);
        else if (key == "height") q.height = (float)scalar(base, key, value);
        else if (key == "N") q.N = integer(base, key, value);
        else if (key == "n") q.n = integer(base, key, value);
        else if (key == "numIterations") q.numIterations = integer(base, key, value);
        else if (key == "maxTreeSize") q.maxTreeSize = integer(base, key, value);
        else if (key == "numDisc") q.numDisc = integer(base, key, value);
        else if (key == "agentLength") q.agentLength = (float)scalar(base, key, value);
        else if (key == "goalThreshold") q.goalThreshold = (float)scalar(base, key, value);
        else if (key == "samplesPerIteration") q.samplesPerIteration = integer(base, key, value);
        else if (key == "device") q.device = integer(base, key, value);
        else if (key == "fixGNewClear") q.fixGNewClear = boolean(key, value);
        else if (key == "batchRule") {
            if (value == "reference") q.batchRule = SBMP_BATCH_REFERENCE;
            else if (value == "fill") q.batchRule = SBMP_BATCH_FILL;
            else throw Error(SBMP_ERR_INVALID_ARGUMENT, "batchRule must be reference or fill");
        } else if (key == "initial" || key == "goal") {
            const std::vector<double> v = numbers_from(base, key, value);
            if (v.size() < 2 || v.size() > 7)
                throw Error(SBMP_ERR_INVALID_ARGUMENT, key + " needs 2 to 7 values (a sample of KGMT.cu:5)");
            float* dst = key == "initial" ? c.initial : c.goal;
            for (int i = 0; i < 7; ++i) dst[i] = i < (int)v.size() ? (float)v[i] : 0.0f;
        } else if (key == "obstacles") {
            const std::string r = resolve(base, value);
            if (r.size() >= sizeof(c.obstacles)) throw Error(SBMP_ERR_INVALID_ARGUMENT, "obstacles path too long");
            strncpy(c.obstacles, r.c_str(), sizeof(c.obstacles) - 1);
        } else if (key == "description") {
        } else {
            throw Error(SBMP_ERR_INVALID_ARGUMENT, p + ":" + std::to_string(lineNo) + ": unknown key '" + key + "'");
        }
    }
    *out = c;
}

}  // namespace sbmp
