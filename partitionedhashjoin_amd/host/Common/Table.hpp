// Relation types of the reference API (src/Common/Table.hpp:20-57), kept
// source-compatible: Tuple {id, payload} is bit-identical to phj_tuple, so a
// Table<Tuple> hands &(*table)[0] / GetSize() straight to the C ABI.
#pragma once

#include <cstdint>
#include <iostream>
#include <string>
#include <vector>

#include "phj.h"

namespace Common {

std::string generate_uuid();

struct alignas(16) Tuple {
    int64_t id;
    int64_t payload;

    friend std::ostream& operator<<(std::ostream& out, const Tuple& t) {
        return out << t.id << ", " << t.payload;
    }
};
static_assert(sizeof(Tuple) == sizeof(phj_tuple), "Tuple must match phj_tuple");

struct JoinedTuple {
    int64_t id;
    int64_t payloadA;
    int64_t payloadB;

    friend std::ostream& operator<<(std::ostream& out, const JoinedTuple& t) {
        return out << t.id << ", " << t.payloadA << ", " << t.payloadB;
    }
};

template <typename TupleType>
class Table {
   public:
    explicit Table(std::string id) : m_id(std::move(id)) {}
    Table(size_t size, std::string id) : m_id(std::move(id)), m_tuples(size) {}

    TupleType& operator[](size_t index) { return m_tuples[index]; }
    const TupleType& operator[](size_t index) const { return m_tuples[index]; }
    size_t GetSize() const { return m_tuples.size(); }
    size_t GetCapacity() const { return m_tuples.capacity(); }
    std::string GetID() const { return m_id; }
    TupleType* Data() { return m_tuples.data(); }
    const TupleType* Data() const { return m_tuples.data(); }

   private:
    const std::string m_id;
    std::vector<TupleType> m_tuples;
};

}  // namespace Common
