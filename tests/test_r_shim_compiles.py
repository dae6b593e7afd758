"""The R `.Call` shim of INTEGRATION.md §2 compiles against include/ppls.h (no GPU, no R).

R is not installed in this image, so the shim cannot be built against R's headers here.  This test
extracts the C block from INTEGRATION.md and type-checks it with gcc against (a) the real
include/ppls.h and (b) a declaration-only list of the R C API prototypes the shim calls, written
from R's documented API ("Writing R Extensions", §5/§6).  It catches wrong argument counts, types
and names of ppls_* calls and structs -- not R runtime behaviour.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

R_API = r"""
#pragma once
#include <stddef.h>
#include <stdint.h>
typedef struct SEXPREC* SEXP;
typedef ptrdiff_t R_xlen_t;
typedef enum { FALSE = 0, TRUE } Rboolean;
typedef unsigned int SEXPTYPE;
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
#define NA_INTEGER (-2147483647 - 1)
extern SEXP R_NilValue;
extern SEXP R_NamesSymbol;
void Rf_error(const char*, ...) __attribute__((noreturn));
void Rf_warning(const char*, ...);
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
void* R_ExternalPtrAddr(SEXP);
void R_ClearExternalPtr(SEXP);
SEXP R_MakeExternalPtr(void*, SEXP, SEXP);
typedef void (*R_CFinalizer_t)(SEXP);
void R_RegisterCFinalizerEx(SEXP, R_CFinalizer_t, Rboolean);
Rboolean Rf_isReal(SEXP);
Rboolean Rf_isMatrix(SEXP);
Rboolean Rf_isNewList(SEXP);
Rboolean Rf_isInteger(SEXP);
Rboolean Rf_isNull(SEXP);
int Rf_nrows(SEXP);
int Rf_ncols(SEXP);
int Rf_length(SEXP);
R_xlen_t XLENGTH(SEXP);
SEXP VECTOR_ELT(SEXP, R_xlen_t);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
void SET_STRING_ELT(SEXP, R_xlen_t, SEXP);
double* REAL(SEXP);
int* INTEGER(SEXP);
int Rf_asInteger(SEXP);
double Rf_asReal(SEXP);
SEXP Rf_duplicate(SEXP);
SEXP Rf_allocVector(SEXPTYPE, R_xlen_t);
SEXP Rf_allocMatrix(SEXPTYPE, int, int);
SEXP Rf_alloc3DArray(SEXPTYPE, int, int, int);
SEXP Rf_ScalarReal(double);
SEXP Rf_ScalarInteger(int);
SEXP Rf_lengthgets(SEXP, R_xlen_t);
SEXP Rf_mkChar(const char*);
SEXP Rf_setAttrib(SEXP, SEXP, SEXP);
char* R_alloc(size_t, int);
"""


def _shim_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2. R `.Call` shim"):]
    m = re.search(r"```c\n(.*?)```", sec, re.S)
    assert m, "no C block in INTEGRATION.md §2"
    return m.group(1)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_r_shim_type_checks(tmp_path):
    src = _shim_source()
    assert "PPLS_gpu_simult" in src and "Expectations" in open(os.path.join(ROOT, "INTEGRATION.md")).read()
    (tmp_path / "R.h").write_text("#pragma once\n")
    (tmp_path / "Rinternals.h").write_text(R_API)
    (tmp_path / "shim.c").write_text(src)
    res = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Werror", "-Wno-unused-function",
                          "-I", str(tmp_path), "-I", os.path.join(ROOT, "include"), str(tmp_path / "shim.c")],
                         capture_output=True, text=True)
    assert res.returncode == 0, res.stderr
