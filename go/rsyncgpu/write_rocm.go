//go:build cgo && rocm

package rsyncgpu

// rsg_write_fn of rsg_generate_files_fd (include/rsg.h): the engine hands each
// batch of the sums stream to the caller's io.Writer through this export.  A
// file with //export may only declare, not define, C functions in its
// preamble, so it lives apart from rsyncgpu_rocm.go.

/*
#include <stdint.h>
*/
import "C"

import (
	"io"
	"runtime/cgo"
	"unsafe"
)

//export rsgGoWrite
func rsgGoWrite(user unsafe.Pointer, data *C.uint8_t, n C.uint64_t) C.int32_t {
	w := (*(*cgo.Handle)(user)).Value().(io.Writer)
	if _, err := w.Write(unsafe.Slice((*byte)(unsafe.Pointer(data)), int(n))); err != nil {
		return -1
	}
	return 0
}
