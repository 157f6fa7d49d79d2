// Filter registry + batched Get filter step (SURVEY.md §8(f) rows 1-2) — additive API beside the
// drop-in bloom.go.  The reference's callers do not use it; a batched MultiGet would:
//
//	OpenSSTable (lsm/sstable.go:121-129)        -> reg.Put(fileNum, level, bloomBlock, minKey, maxKey)
//	compaction removes inputs (compaction.go:335-343) -> reg.Remove(fileNum)
//	LSM.Get's walk + MayContain (lsm/lsm.go:168-198) -> reg.Candidates(keys)
//
// Not compiled in this repository's pipeline (no Go toolchain in the image); the C ABI it calls is
// tested through the Python binding (tests/test_gpu_parity.py, test_registry_*).
package lsm

/*
#include <stdint.h>
#include <stdlib.h>
#include "seb_bloom.h"
*/
import "C"

import (
	"runtime"
	"sync/atomic"
	"unsafe"
)

// FilterRegistry holds the bloom filters of the open SSTables in HBM (one per LSM instance).
type FilterRegistry struct {
	h       *C.seb_registry
	capHint atomic.Uint32 // row width of the last Candidates call (the C side re-checks it)
}

func regPanic(op string) {
	panic("lsm: FilterRegistry." + op + ": " + C.GoString(C.seb_last_error()))
}

// NewFilterRegistry creates an empty registry on GPU `device`.
func NewFilterRegistry(device int) *FilterRegistry {
	h := C.seb_registry_new(C.int(device))
	if h == nil {
		regPanic("New")
	}
	r := &FilterRegistry{h: h}
	runtime.SetFinalizer(r, func(r *FilterRegistry) { C.seb_registry_free(r.h) })
	return r
}

func bytesPtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// Put registers an SSTable's bloom block (its Encode() bytes) with the file's level and key
// range; levels 1..4 are kept by MinKey as lsm/levels.go:45-63 keeps them.  Returns the slot.
func (r *FilterRegistry) Put(fileNum uint64, level int, bloomBlock []byte, minKey, maxKey string) int {
	mn, mx := []byte(minKey), []byte(maxKey)
	rc := C.seb_registry_put(r.h, C.uint64_t(fileNum), C.int(level), bytesPtr(bloomBlock), C.uint64_t(len(bloomBlock)),
		bytesPtr(mn), C.uint64_t(len(mn)), bytesPtr(mx), C.uint64_t(len(mx)))
	if rc < 0 {
		regPanic("Put")
	}
	runtime.KeepAlive(bloomBlock)
	return int(rc)
}

// Remove frees a file's filter (compaction deleted the file).
func (r *FilterRegistry) Remove(fileNum uint64) {
	if C.seb_registry_remove(r.h, C.uint64_t(fileNum)) != 0 {
		regPanic("Remove")
	}
}

// Candidates returns, per key, the file numbers Get would read for it — every L0 file and the
// covering file of each level 1..4 whose bloom filter may contain the key — in Get's visiting
// order.  One GPU launch for the whole batch, any number of registered files.
func (r *FilterRegistry) Candidates(keys []string) [][]uint64 {
	out := make([][]uint64, len(keys))
	if len(keys) == 0 {
		return out
	}
	data, offs := packKeys(keys)
	// the seb_keys struct holds Go pointers: it lives in C memory and what it points to is pinned
	var pin runtime.Pinner
	defer pin.Unpin()
	pin.Pin(&data[0])
	pin.Pin(&offs[0])
	ks := (*C.seb_keys)(C.malloc(C.size_t(unsafe.Sizeof(C.seb_keys{}))))
	defer C.free(unsafe.Pointer(ks))
	*ks = C.seb_keys{data: (*C.uint8_t)(unsafe.Pointer(&data[0])), offsets: (*C.uint64_t)(unsafe.Pointer(&offs[0])),
		n: C.uint64_t(len(keys))}
	// One C call sizes the rows, runs the lookup and maps slots to file numbers under the
	// registry's lock, so a concurrent flush (Put) or compaction (Remove + Put reusing the slot)
	// cannot overflow a row or make a slot name the wrong file.  SEB_ERR_RANGE: the registry
	// grew since the last call; retry with the width it reports.
	capRow := C.uint32_t(r.capHint.Load())
	if capRow == 0 {
		capRow = 1
	}
	var files []uint64
	for {
		files = make([]uint64, len(keys)*int(capRow))
		var need C.uint32_t
		rc := C.seb_registry_multiget_files(r.h, ks, (*C.uint64_t)(unsafe.Pointer(&files[0])), capRow, &need)
		if rc == C.int(C.SEB_ERR_RANGE) && need > capRow {
			capRow = need
			continue
		}
		if rc != 0 {
			regPanic("Candidates")
		}
		r.capHint.Store(uint32(capRow))
		break
	}
	runtime.KeepAlive(data)
	runtime.KeepAlive(offs)
	w := int(capRow)
	for i := range keys {
		for _, f := range files[i*w : (i+1)*w] {
			if f == ^uint64(0) {
				break
			}
			out[i] = append(out[i], f)
		}
	}
	return out
}

// packKeys lays keys out as one byte buffer + len(keys)+1 offsets (the seb_keys var-length form).
func packKeys(keys []string) ([]byte, []uint64) {
	total := 0
	for _, k := range keys {
		total += len(k)
	}
	data := make([]byte, total+1)
	offs := make([]uint64, len(keys)+1)
	pos := 0
	for i, k := range keys {
		offs[i] = uint64(pos)
		pos += copy(data[pos:], k)
	}
	offs[len(keys)] = uint64(pos)
	return data, offs
}
