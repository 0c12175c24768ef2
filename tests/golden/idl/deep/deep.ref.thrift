
namespace go deep

enum FOO {
    B,
    A,
}

const string ConstString = "const string"

struct TestStruct {
    1: i64 a
    2: string b
}