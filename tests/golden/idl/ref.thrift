namespace go ref

enum FOO {
    B,
    A,
}

const string ConstString = "const string"
