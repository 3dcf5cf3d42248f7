// sqlite_min.h -- the handful of SQLite C-API entry points the loader uses,
// declared against the system libsqlite3.so.0 (the image ships the shared
// library but no development header).  Signatures and constants are the
// stable public SQLite 3 ABI.
#pragma once
#include <cstdint>

// (a translation unit that already has the real sqlite3.h -- the reference's
// main.cpp, which includes the drop-in adapter after it -- takes its
// declarations and macros instead)
#ifndef SQLITE3_H
extern "C" {
struct sqlite3;
struct sqlite3_stmt;

int sqlite3_open_v2(const char* filename, sqlite3** ppDb, int flags, const char* zVfs);
int sqlite3_close(sqlite3*);
int sqlite3_prepare_v2(sqlite3* db, const char* zSql, int nByte, sqlite3_stmt** ppStmt, const char** pzTail);
int sqlite3_step(sqlite3_stmt*);
int sqlite3_finalize(sqlite3_stmt* pStmt);
int sqlite3_bind_int(sqlite3_stmt*, int, int);
int sqlite3_bind_double(sqlite3_stmt*, int, double);
int sqlite3_bind_text(sqlite3_stmt*, int, const char*, int, void (*)(void*));
int sqlite3_bind_blob(sqlite3_stmt*, int, const void*, int, void (*)(void*));
int sqlite3_reset(sqlite3_stmt* pStmt);
int sqlite3_column_int(sqlite3_stmt*, int iCol);
double sqlite3_column_double(sqlite3_stmt*, int iCol);
const void* sqlite3_column_blob(sqlite3_stmt*, int iCol);
int sqlite3_column_bytes(sqlite3_stmt*, int iCol);
const unsigned char* sqlite3_column_text(sqlite3_stmt*, int iCol);
const char* sqlite3_errmsg(sqlite3*);
const char* sqlite3_errstr(int);
int sqlite3_exec(sqlite3*, const char* sql, int (*callback)(void*, int, char**, char**), void*, char** errmsg);
}

constexpr int SQLITE_OK = 0;
constexpr int SQLITE_ROW = 100;
constexpr int SQLITE_DONE = 101;
constexpr int SQLITE_OPEN_READONLY = 0x00000001;
constexpr int SQLITE_OPEN_URI = 0x00000040;
constexpr int SQLITE_OPEN_READWRITE = 0x00000002;
constexpr int SQLITE_OPEN_CREATE = 0x00000004;
#endif
#define PFAAI_SQLITE_TRANSIENT (reinterpret_cast<void (*)(void*)>(-1))
