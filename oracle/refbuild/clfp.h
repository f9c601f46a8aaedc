#pragma OPENCL EXTENSION __cl_clang_function_pointers : enable
