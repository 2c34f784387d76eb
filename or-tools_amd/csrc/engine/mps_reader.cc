// MPS ingestion for the engine's C ABI (include/mi_lp.h, mi_mps_*), a
// from-scratch restatement of OR-Tools 9.7's reader with the LinearProgram
// data wrapper:
//   ortools/lp_data/mps_reader_template.h   sections, fields, bound and row
//                                           semantics (MPSReaderTemplate)
//   ortools/lp_data/mps_reader_template.cc  fixed-format columns, line checks
//   ortools/lp_data/mps_reader.cc:22-112    DataWrapper<LinearProgram>
//   ortools/lp_data/lp_data.cc:164-205      new variables [0, +inf), new
//                                           constraints [0, 0]
// Same acceptance rules (auto-detection tries fixed, then free format), same
// resulting bounds, objective, offset and matrix (columns cleaned up: sorted
// rows, zeros dropped, the last of duplicate entries kept). Integer markers
// are parsed (0/1 default bounds, as upstream); the LP is their relaxation.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/mi_lp.h"
#include "lp_data.h"

struct mi_mps_model {
  std::string name;
  bool maximize = false;
  double objective_offset = 0.0;
  std::vector<double> objective;
  std::vector<double> col_lb, col_ub;
  std::vector<int8_t> is_integer;
  std::vector<double> row_lb, row_ub;
  std::vector<milp::SparseColumn> columns;
  std::vector<std::string> col_names, row_names;
  std::string error;
};

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();
constexpr int kNumFields = 6;
// mps_reader_template.cc: fixed-format field columns and the blanks between.
constexpr int kFieldStart[kNumFields] = {1, 4, 14, 24, 39, 49};
constexpr int kFieldLength[kNumFields] = {2, 8, 8, 12, 8, 12};
constexpr int kSpacePos[12] = {12, 13, 22, 23, 36, 37, 38, 47, 48, 61, 62, 63};

enum class Section {
  kUnknown, kName, kObjsense, kRows, kLazycons, kColumns, kRhs, kRanges, kBounds,
  kIndicators, kEndData
};
enum class RowType { kEquality, kLessThan, kGreaterThan, kNone };
enum class BoundType { kLower, kUpper, kFixed, kFree, kMinusInf, kPlusInf, kBinary, kSemi };

struct ParseError {
  std::string message;
};

std::string StripTrailing(const std::string& s) {
  size_t e = s.size();
  while (e > 0 && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r' || s[e - 1] == '\n'))
    --e;
  return s.substr(0, e);
}

std::vector<std::string> SplitFree(const std::string& line) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < line.size()) {
    while (i < line.size() && (line[i] == ' ' || line[i] == '\t')) ++i;
    if (i >= line.size()) break;
    size_t j = i;
    while (j < line.size() && line[j] != ' ' && line[j] != '\t') ++j;
    out.push_back(line.substr(i, j - i));
    i = j;
  }
  return out;
}

// internal::MPSLineInfo
struct Line {
  int64_t number = 0;
  bool free_form = true;
  std::string text;
  std::vector<std::string> fields;

  bool IsCommentOrBlank() const { return text.empty() || text[0] == '*'; }
  bool IsNewSection() const { return !text.empty() && text[0] != ' '; }
  std::string FirstWord() const { return text.substr(0, text.find(' ')); }
  int FieldOffset() const { return free_form ? static_cast<int>(fields.size() & 1) : 0; }
  bool IsFixedFormat() const {
    const int max_size = kFieldStart[kNumFields - 1] + kFieldLength[kNumFields - 1];
    const int size = static_cast<int>(text.size());
    if (size > max_size) return false;
    for (const int p : kSpacePos) {
      if (p >= size) break;
      if (text[p] != ' ') return false;
    }
    return true;
  }
  [[noreturn]] void Fail(const std::string& what) const {
    throw ParseError{what + " Line " + std::to_string(number) + ": \"" + text + "\"."};
  }
};

Line MakeLine(int64_t number, bool free_form, const std::string& raw) {
  Line l;
  l.number = number;
  l.free_form = free_form;
  l.text = StripTrailing(raw);
  if (!free_form && l.text.find('\t') != std::string::npos) l.Fail("File contains tabs.");
  if (l.IsCommentOrBlank()) return l;
  if (free_form) {
    l.fields = SplitFree(l.text);
    if (l.fields.size() > static_cast<size_t>(kNumFields)) l.Fail("Found too many fields.");
  } else {
    const int size = static_cast<int>(l.text.size());
    for (int i = 0; i < kNumFields; ++i) {
      if (kFieldStart[i] >= size) break;
      l.fields.push_back(StripTrailing(l.text.substr(kFieldStart[i], kFieldLength[i])));
    }
  }
  return l;
}

// absl::SimpleAtod: surrounding whitespace allowed, the whole token parsed.
double ParseDouble(const std::string& s, const Line& line) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  const std::string t = s.substr(b, e - b);
  if (t.empty()) line.Fail("Failed to convert \"" + s + "\" to double.");
  char* end = nullptr;
  errno = 0;
  double v = std::strtod(t.c_str(), &end);
  if (end != t.c_str() + t.size()) line.Fail("Failed to convert \"" + s + "\" to double.");
  if (std::isnan(v)) line.Fail("Found NaN value.");
  return v;
}

class Reader {
 public:
  Reader(bool free_form, mi_mps_model* data) : free_form_(free_form), data_(data) {
    *data_ = mi_mps_model();
  }

  void Process(int64_t number, const std::string& raw) {
    const Line line = MakeLine(number, free_form_, raw);
    if (line.IsCommentOrBlank()) return;
    if (line.IsNewSection()) {
      static const std::unordered_map<std::string, Section> kSections = {
          {"NAME", Section::kName},       {"OBJSENSE", Section::kObjsense},
          {"ROWS", Section::kRows},       {"LAZYCONS", Section::kLazycons},
          {"COLUMNS", Section::kColumns}, {"RHS", Section::kRhs},
          {"RANGES", Section::kRanges},   {"BOUNDS", Section::kBounds},
          {"INDICATORS", Section::kIndicators}, {"ENDATA", Section::kEndData}};
      const auto it = kSections.find(line.FirstWord());
      if (it == kSections.end()) line.Fail("Unknown section.");
      section_ = it->second;
      if (!free_form_ && !line.IsFixedFormat() && section_ != Section::kName) {
        line.Fail("Line is not in fixed format.");
      }
      if (section_ == Section::kName) {
        if (free_form_) {
          if (line.fields.size() >= 2) data_->name = line.fields[1];
        } else {
          const std::vector<std::string> free_fields = SplitFree(line.text);
          const std::string free_name = free_fields.size() >= 2 ? free_fields[1] : "";
          const std::string fixed_name = line.fields.size() >= 3 ? line.fields[2] : "";
          if (free_name != fixed_name) {
            line.Fail("Fixed form invalid: name differs between free and fixed forms.");
          }
          data_->name = fixed_name;
        }
      }
      return;
    }
    if (!free_form_ && !line.IsFixedFormat()) line.Fail("Line is not in fixed format.");
    switch (section_) {
      case Section::kName:
        line.Fail("Second NAME field.");
      case Section::kObjsense: {
        const std::vector<std::string> w = SplitFree(line.text);
        const std::string field = w.size() == 1 ? w[0] : std::string("?");
        if (field != "MIN" && field != "MAX") line.Fail("Expected objective sense (MAX or MIN).");
        data_->maximize = (field == "MAX");
        return;
      }
      case Section::kRows:
      case Section::kLazycons:
        return Rows(line);
      case Section::kColumns:
        return Columns(line);
      case Section::kRhs:
        return RhsOrRanges(line, /*ranges=*/false);
      case Section::kRanges:
        return RhsOrRanges(line, /*ranges=*/true);
      case Section::kBounds:
        return Bounds(line);
      case Section::kIndicators:
        // DataWrapper<LinearProgram>::CreateIndicatorConstraint.
        line.Fail("LinearProgram does not support indicator constraints.");
      case Section::kEndData:
        return;
      default:
        line.Fail("Unknown section.");
    }
  }

  // LinearProgram::CleanUp: each column sorted by row, zeros dropped, the last
  // of duplicate entries kept (SparseVector::CleanUp).
  void Finish() {
    for (milp::SparseColumn& c : data_->columns) c.CleanUp();
  }

 private:
  int FindOrCreateConstraint(const std::string& name) {
    const auto it = row_index_.find(name);
    if (it != row_index_.end()) return it->second;
    const int row = static_cast<int>(data_->row_lb.size());
    row_index_.emplace(name, row);
    data_->row_lb.push_back(0.0);
    data_->row_ub.push_back(0.0);
    data_->row_names.push_back(name);
    return row;
  }
  int FindOrCreateVariable(const std::string& name) {
    const auto it = col_index_.find(name);
    if (it != col_index_.end()) return it->second;
    const int col = static_cast<int>(data_->col_lb.size());
    col_index_.emplace(name, col);
    data_->objective.push_back(0.0);
    data_->col_lb.push_back(0.0);
    data_->col_ub.push_back(kInf);
    data_->is_integer.push_back(0);
    data_->columns.emplace_back();
    data_->col_names.push_back(name);
    return col;
  }

  void Rows(const Line& line) {
    if (line.fields.size() < 2) line.Fail("Not enough fields in ROWS section.");
    const std::string& type_name = line.fields[0];
    const std::string& row_name = line.fields[1];
    RowType type;
    if (type_name == "E") type = RowType::kEquality;
    else if (type_name == "L") type = RowType::kLessThan;
    else if (type_name == "G") type = RowType::kGreaterThan;
    else if (type_name == "N") type = RowType::kNone;
    else line.Fail("Unknown row type.");
    if (objective_name_.empty() && type == RowType::kNone) {
      objective_name_ = row_name;
      return;
    }
    const int row = FindOrCreateConstraint(row_name);
    switch (type) {
      case RowType::kLessThan:
        data_->row_lb[row] = -kInf;
        break;
      case RowType::kGreaterThan:
        data_->row_ub[row] = kInf;
        break;
      case RowType::kNone:
        data_->row_lb[row] = -kInf;
        data_->row_ub[row] = kInf;
        break;
      case RowType::kEquality:
        break;
    }
  }

  void StoreCoefficient(const Line& line, int col, const std::string& row_name,
                        const std::string& row_value) {
    if (row_name.empty() || row_name == "$") return;
    const double value = ParseDouble(row_value, line);
    if (value == kInf || value == -kInf) line.Fail("Constraint coefficients cannot be infinity.");
    if (value == 0.0) return;
    if (row_name == objective_name_) {
      data_->objective[col] = value;
    } else {
      const int row = FindOrCreateConstraint(row_name);
      data_->columns[col].SetCoefficient(row, value);
    }
  }

  void Columns(const Line& line) {
    if (line.text.find("'MARKER'") != std::string::npos) {
      if (line.text.find("'INTORG'") != std::string::npos) {
        if (in_integer_section_) line.Fail("Found INTORG inside the integer section.");
        in_integer_section_ = true;
      } else if (line.text.find("'INTEND'") != std::string::npos) {
        if (!in_integer_section_) line.Fail("Found INTEND without corresponding INTORG.");
        in_integer_section_ = false;
      }
      return;
    }
    const size_t start = free_form_ ? 0 : 1;
    if (line.fields.size() < start + 3) line.Fail("Not enough fields in COLUMNS section.");
    const int col = FindOrCreateVariable(line.fields[start]);
    if (binary_by_default_.size() < static_cast<size_t>(col) + 1) {
      binary_by_default_.resize(col + 1, false);
    }
    if (in_integer_section_) {
      data_->is_integer[col] = 1;
      data_->col_lb[col] = 0.0;
      data_->col_ub[col] = 1.0;
      binary_by_default_[col] = true;
    } else {
      data_->col_lb[col] = 0.0;
      data_->col_ub[col] = kInf;
    }
    StoreCoefficient(line, col, line.fields[start + 1], line.fields[start + 2]);
    if (line.fields.size() == start + 4) line.Fail("Unexpected number of fields.");
    if (line.fields.size() - start > 4) {
      StoreCoefficient(line, col, line.fields[start + 3], line.fields[start + 4]);
    }
  }

  void StoreRhs(const Line& line, const std::string& row_name, const std::string& value_text) {
    if (row_name.empty()) return;
    if (row_name != objective_name_) {
      const int row = FindOrCreateConstraint(row_name);
      const double value = ParseDouble(value_text, line);
      data_->row_lb[row] = data_->row_lb[row] == -kInf ? -kInf : value;
      data_->row_ub[row] = data_->row_ub[row] == kInf ? kInf : value;
    } else {
      data_->objective_offset = -ParseDouble(value_text, line);
    }
  }

  void StoreRange(const Line& line, const std::string& row_name, const std::string& value_text) {
    if (row_name.empty()) return;
    const int row = FindOrCreateConstraint(row_name);
    const double range = ParseDouble(value_text, line);
    double lb = data_->row_lb[row];
    double ub = data_->row_ub[row];
    if (lb == ub) {
      if (range < 0.0) {
        lb += range;
      } else {
        ub += range;
      }
    }
    if (lb == -kInf) lb = ub - std::fabs(range);
    if (ub == kInf) ub = lb + std::fabs(range);
    data_->row_lb[row] = lb;
    data_->row_ub[row] = ub;
  }

  void RhsOrRanges(const Line& line, bool ranges) {
    const size_t start = free_form_ ? 0 : 2;
    const size_t offset = start + line.FieldOffset();
    if (line.fields.size() < offset + 2) line.Fail("Not enough fields in RHS section.");
    auto store = [&](const std::string& name, const std::string& value) {
      if (ranges) {
        StoreRange(line, name, value);
      } else {
        StoreRhs(line, name, value);
      }
    };
    store(line.fields[offset], line.fields[offset + 1]);
    if (line.fields.size() >= start + 4) {
      if (line.fields.size() < offset + 4) line.Fail("Not enough fields in RHS section.");
      store(line.fields[offset + 2], line.fields[offset + 3]);
    }
  }

  void Bounds(const Line& line) {
    if (line.fields.size() < 3) line.Fail("Not enough fields in BOUNDS section.");
    const std::string& mnemonic = line.fields[0];
    const std::string& column_name = line.fields[2];
    const std::string value_text = line.fields.size() >= 4 ? line.fields[3] : "";
    static const std::unordered_map<std::string, BoundType> kBounds = {
        {"LO", BoundType::kLower}, {"UP", BoundType::kUpper},    {"FX", BoundType::kFixed},
        {"FR", BoundType::kFree},  {"MI", BoundType::kMinusInf}, {"PL", BoundType::kPlusInf},
        {"BV", BoundType::kBinary}, {"LI", BoundType::kLower},   {"UI", BoundType::kUpper},
        {"SC", BoundType::kSemi}};
    const auto it = kBounds.find(mnemonic);
    if (it == kBounds.end()) line.Fail("Unknown bound type.");
    const int col = FindOrCreateVariable(column_name);
    if (mnemonic == "BV" || mnemonic == "LI" || mnemonic == "UI") data_->is_integer[col] = 1;
    if (binary_by_default_.size() <= static_cast<size_t>(col)) {
      binary_by_default_.resize(col + 1, false);
    }
    double lb = data_->col_lb[col];
    double ub = data_->col_ub[col];
    if (binary_by_default_[col]) {
      lb = 0.0;
      ub = kInf;
    }
    switch (it->second) {
      case BoundType::kLower:
        lb = ParseDouble(value_text, line);
        if (mnemonic == "LI" && lb == 0.0) ub = kInf;
        break;
      case BoundType::kUpper:
        ub = ParseDouble(value_text, line);
        break;
      case BoundType::kSemi:
        // DataWrapper<LinearProgram>::SetVariableTypeToSemiContinuous is fatal.
        line.Fail("Semi continuous variables are not supported.");
      case BoundType::kFixed:
        lb = ParseDouble(value_text, line);
        ub = lb;
        break;
      case BoundType::kFree:
        lb = -kInf;
        ub = kInf;
        break;
      case BoundType::kMinusInf:
        lb = -kInf;
        break;
      case BoundType::kPlusInf:
        ub = kInf;
        break;
      case BoundType::kBinary:
        lb = 0.0;
        ub = 1.0;
        break;
    }
    binary_by_default_[col] = false;
    data_->col_lb[col] = lb;
    data_->col_ub[col] = ub;
  }

  bool free_form_;
  mi_mps_model* data_;
  Section section_ = Section::kUnknown;
  std::string objective_name_;
  bool in_integer_section_ = false;
  std::vector<bool> binary_by_default_;
  std::unordered_map<std::string, int> row_index_;
  std::unordered_map<std::string, int> col_index_;
};

// MPSReaderTemplate::ParseString / ParseFile for one explicit format.
bool ParseText(const std::string& text, bool free_form, mi_mps_model* out) {
  Reader reader(free_form, out);
  try {
    std::istringstream in(text);
    std::string raw;
    int64_t number = 0;
    while (std::getline(in, raw)) reader.Process(++number, raw);
    reader.Finish();
  } catch (const ParseError& e) {
    const std::string message = e.message;
    *out = mi_mps_model();
    out->error = message;
    return false;
  }
  return true;
}

int Parse(const std::string& text, int32_t format, mi_mps_model* model, int32_t* used) {
  if (format == MI_MPS_FIXED || format == MI_MPS_FREE) {
    const bool ok = ParseText(text, format == MI_MPS_FREE, model);
    if (used != nullptr) *used = format;
    return ok ? MI_LP_OK : MI_LP_ERROR_INVALID_PROBLEM;
  }
  // Auto-detection: fixed format first, then free (mps_reader_template.h).
  if (ParseText(text, false, model)) {
    if (used != nullptr) *used = MI_MPS_FIXED;
    return MI_LP_OK;
  }
  const bool ok = ParseText(text, true, model);
  if (used != nullptr) *used = MI_MPS_FREE;
  return ok ? MI_LP_OK : MI_LP_ERROR_INVALID_PROBLEM;
}

}  // namespace

extern "C" {

int mi_mps_parse_string(const char* text, int32_t format, mi_mps_model** out,
                        int32_t* format_used) {
  if (text == nullptr || out == nullptr) return MI_LP_ERROR_NULL;
  mi_mps_model* model = new mi_mps_model();
  const int rc = Parse(std::string(text), format, model, format_used);
  *out = model;
  return rc;
}

int mi_mps_read_file(const char* path, int32_t format, mi_mps_model** out,
                     int32_t* format_used) {
  if (path == nullptr || out == nullptr) return MI_LP_ERROR_NULL;
  std::ifstream f(path, std::ios::binary);
  mi_mps_model* model = new mi_mps_model();
  *out = model;
  if (!f) {
    model->error = std::string("Cannot open file: ") + path;
    return MI_LP_ERROR_INVALID_PROBLEM;
  }
  std::ostringstream ss;
  ss << f.rdbuf();
  return Parse(ss.str(), format, model, format_used);
}

const char* mi_mps_error(const mi_mps_model* m) {
  return m == nullptr ? "null model" : m->error.c_str();
}

int mi_mps_dims(const mi_mps_model* m, int32_t* num_rows, int32_t* num_cols, int64_t* nnz) {
  if (m == nullptr) return MI_LP_ERROR_NULL;
  if (num_rows) *num_rows = static_cast<int32_t>(m->row_lb.size());
  if (num_cols) *num_cols = static_cast<int32_t>(m->col_lb.size());
  if (nnz) {
    int64_t n = 0;
    for (const milp::SparseColumn& c : m->columns) n += c.num_entries();
    *nnz = n;
  }
  return MI_LP_OK;
}

int mi_mps_get(const mi_mps_model* m, int64_t* col_starts, int32_t* row_idx, double* vals,
               double* col_lb, double* col_ub, double* row_lb, double* row_ub, double* obj,
               double* obj_offset, int32_t* maximize, int8_t* is_integer) {
  if (m == nullptr) return MI_LP_ERROR_NULL;
  const size_t n = m->col_lb.size();
  int64_t k = 0;
  for (size_t j = 0; j < n; ++j) {
    if (col_starts) col_starts[j] = k;
    const milp::SparseColumn& c = m->columns[j];
    for (int64_t i = 0; i < c.num_entries(); ++i, ++k) {
      if (row_idx) row_idx[k] = c.rows[i];
      if (vals) vals[k] = c.coefs[i];
    }
  }
  if (col_starts) col_starts[n] = k;
  for (size_t j = 0; j < n; ++j) {
    if (col_lb) col_lb[j] = m->col_lb[j];
    if (col_ub) col_ub[j] = m->col_ub[j];
    if (obj) obj[j] = m->objective[j];
    if (is_integer) is_integer[j] = m->is_integer[j];
  }
  for (size_t i = 0; i < m->row_lb.size(); ++i) {
    if (row_lb) row_lb[i] = m->row_lb[i];
    if (row_ub) row_ub[i] = m->row_ub[i];
  }
  if (obj_offset) *obj_offset = m->objective_offset;
  if (maximize) *maximize = m->maximize ? 1 : 0;
  return MI_LP_OK;
}

const char* mi_mps_name(const mi_mps_model* m) { return m == nullptr ? "" : m->name.c_str(); }

const char* mi_mps_col_name(const mi_mps_model* m, int32_t col) {
  if (m == nullptr || col < 0 || static_cast<size_t>(col) >= m->col_names.size()) return "";
  return m->col_names[col].c_str();
}

const char* mi_mps_row_name(const mi_mps_model* m, int32_t row) {
  if (m == nullptr || row < 0 || static_cast<size_t>(row) >= m->row_names.size()) return "";
  return m->row_names[row].c_str();
}

void mi_mps_free(mi_mps_model* m) { delete m; }

}  // extern "C"
