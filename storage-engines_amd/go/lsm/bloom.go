// Package lsm — drop-in replacement for intellect4all/storage-engines lsm/bloom.go.
//
// Same exported API, same semantics, bit-exact results; the filter's bit array lives in MI355X
// HBM and is built / probed by hand-written gfx950 kernels in libseb_bloom.so (C ABI:
// include/seb_bloom.h).  The callers — lsm/sstable_builder.go:30,53,217 (NewBloomFilter, Add,
// Encode) and lsm/sstable.go:129,206 (DecodeBloomFilter, MayContain) — compile unchanged.
//
// Not compiled in this repository's pipeline: no Go toolchain exists in the build image or on
// the GPU box (see DESIGN.md).  storage-engines_amd/harness/sstable_replay.c exercises the identical C call sequence.
//
// Build: copy this file over lsm/bloom.go, point the cgo flags at the checkout, `go build`.
package lsm

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../lib -lseb_bloom -Wl,-rpath,${SRCDIR}/../../lib
#include <stdint.h>
#include <stdlib.h>
#include "seb_bloom.h"
*/
import "C"

import (
	"runtime"
	"unsafe"
)

// BloomFilter is a probabilistic data structure for membership testing.
// (lsm/bloom.go:10-14: bits, numBits, numHashes — held by the library, in HBM.)
type BloomFilter struct {
	h *C.seb_filter
}

func libPanic(op string) {
	panic("lsm: BloomFilter." + op + ": " + C.GoString(C.seb_last_error()))
}

func wrap(h *C.seb_filter) *BloomFilter {
	bf := &BloomFilter{h: h}
	runtime.SetFinalizer(bf, func(b *BloomFilter) { C.seb_filter_free(b.h) })
	return bf
}

// NewBloomFilter creates a new bloom filter with optimal parameters (lsm/bloom.go:19).
// expectedKeys: estimated number of keys to insert
// falsePositiveRate: desired false positive rate (e.g., 0.01 for 1%)
func NewBloomFilter(expectedKeys int, falsePositiveRate float64) *BloomFilter {
	h := C.seb_filter_new(C.int64_t(expectedKeys), C.double(falsePositiveRate))
	if h == nil {
		libPanic("New")
	}
	return wrap(h)
}

func strPtr(s string) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(unsafe.StringData(s)))
}

// Add inserts a key into the bloom filter (lsm/bloom.go:70).  The key bytes are copied into the
// filter's pending batch; the bits are set on the GPU in one launch at the next Encode /
// MayContain (the SSTable builder calls Add once per sorted entry, then Encode at Finish).
func (bf *BloomFilter) Add(key string) {
	if C.seb_filter_add(bf.h, strPtr(key), C.uint64_t(len(key))) != 0 {
		libPanic("Add")
	}
	runtime.KeepAlive(key)
}

// MayContain checks if a key might be in the set (lsm/bloom.go:82).
// Returns true if the key might be present (or false positive)
// Returns false if the key is definitely not present
func (bf *BloomFilter) MayContain(key string) bool {
	rc := C.seb_filter_may_contain(bf.h, strPtr(key), C.uint64_t(len(key)))
	runtime.KeepAlive(key)
	if rc < 0 {
		libPanic("MayContain")
	}
	return rc == 1
}

// MayContainBatch answers MayContain for many keys in one GPU launch (additive API; a batched
// LSM MultiGet is the intended caller).  out must have len(keys) elements.
func (bf *BloomFilter) MayContainBatch(keys []string, out []bool) {
	if len(out) < len(keys) {
		panic("lsm: MayContainBatch: out too short")
	}
	if len(keys) == 0 {
		return
	}
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
	kb := C.seb_keys{
		data:    (*C.uint8_t)(unsafe.Pointer(&data[0])),
		offsets: (*C.uint64_t)(unsafe.Pointer(&offs[0])),
		n:       C.uint64_t(len(keys)),
	}
	// Go's bool is one byte holding 0 or 1: the library writes exactly that.
	if C.seb_filter_may_contain_batch(bf.h, &kb, (*C.uint8_t)(unsafe.Pointer(&out[0]))) != 0 {
		libPanic("MayContainBatch")
	}
	runtime.KeepAlive(data)
	runtime.KeepAlive(offs)
}

// Encode serializes the bloom filter to bytes (lsm/bloom.go:96).
// Format: [numBits(8)][numHashes(4)][bits...]
func (bf *BloomFilter) Encode() []byte {
	n := C.seb_filter_encoded_size(bf.h)
	buf := make([]byte, int(n))
	if C.seb_filter_encode(bf.h, (*C.uint8_t)(unsafe.Pointer(&buf[0])), n) != 0 {
		libPanic("Encode")
	}
	return buf
}

// DecodeBloomFilter deserializes a bloom filter from bytes (lsm/bloom.go:105).
func DecodeBloomFilter(data []byte) *BloomFilter {
	if len(data) < 12 {
		return nil
	}
	h := C.seb_filter_decode((*C.uint8_t)(unsafe.Pointer(&data[0])), C.uint64_t(len(data)))
	runtime.KeepAlive(data)
	if h == nil {
		return nil
	}
	return wrap(h)
}
