// Package contivcls binds the MI355X batched first-match ACL classifier
// (include/contivcls.h, vpp_amd/libcontivcls.so) for the Contiv-VPP Go host.
//
// It is a drop-in for mock/aclengine.MockACLEngine
// (mock/aclengine/aclengine_mock.go:94-728): the same method set, the same
// verdict enums, the same error behaviour, with the ACL evaluation moved to
// the GPU and two batched entry points added (ClassifyBatch, ConnectionBatch).
//
// UNTESTED: the build image of this repository has no Go toolchain (SURVEY
// 8(c)), so this file has never been compiled.  The Python host
// (vpp_amd/engine.py, class ACLEngine) calls exactly the same C symbols in
// the same order and is what the parity tests exercise; keep the two in step.
//
// Go 1.9 (the reference's toolchain, .travis.yml:7-8): no runtime.Pinner,
// no unsafe.Slice, no post-1.9 library call.  Ownership (cgo rule): every
// pointer handed to the C ABI is valid only for the duration of the call;
// the engine deep-copies rules and keeps no caller pointer.  Packet and
// connection arrays go to the static C shims of include/contivcls_go.h as
// one scalar pointer per slice (pointer-free Go memory, which cgo allows for
// the call), and the shims build the ABI's SoA records on the C stack -- a
// Go value holding Go pointers never crosses.  Rule records hold only C
// strings (C.CString).  The shims themselves run on the GPU in
// tests/test_gpu_go_shims.py (go/shimtest/shimtest.c, gcc).
package contivcls

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../vpp_amd -lcontivcls -Wl,-rpath,${SRCDIR}/../../vpp_amd
#include <stdlib.h>
#include "contivcls_go.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"net"
	"strings"
	"sync"
	"unsafe"

	"github.com/contiv/vpp/mock/aclengine"
	"github.com/contiv/vpp/mock/localclient"
	"github.com/contiv/vpp/plugins/contiv"
	podmodel "github.com/contiv/vpp/plugins/ksr/model/pod"
	vpp_acl "github.com/ligato/vpp-agent/plugins/defaultplugins/common/model/acl"
)

// ACLAction values of evalACL (aclengine_mock.go:63-77) as the C ABI returns
// them per packet.
const (
	ACLDeny    = uint8(C.CLS_ACL_DENY)
	ACLPermit  = uint8(C.CLS_ACL_PERMIT)
	ACLReflect = uint8(C.CLS_ACL_REFLECT)
	ACLFailure = uint8(C.CLS_ACL_FAILURE)
)

// Engine replaces MockACLEngine.  The Go side keeps the pod registry and the
// installed protobufs (DumpACLs returns them); interface bindings and the
// compiled tables live in the C engine.
type Engine struct {
	sync.Mutex
	e      *C.cls_engine
	Contiv contiv.API

	pods   map[podmodel.ID]*podConfig
	byName map[string]*vpp_acl.AccessLists_Acl
}

type podConfig struct {
	ip          net.IP
	anotherNode bool
}

// New replaces NewMockACLEngine (aclengine_mock.go:124).  device: HIP device
// ordinal, -1 for the current one.
func New(c contiv.API, device int) (*Engine, error) {
	return NewMulti(c, []int{device})
}

// NewMulti: one engine over several devices (SURVEY 8(e)).  Every table is
// compiled once and replicated to every device; Batch packets shard over the
// devices; over distinct devices the hit counters of ClassifyBatchDevice are
// merged by the library's RCCL all-reduce over xGMI.
func NewMulti(c contiv.API, devices []int) (*Engine, error) {
	// the library this binding was written against (include/contivcls.h)
	if v := C.cls_abi_version(); v != C.clsg_abi_version() {
		return nil, fmt.Errorf("contivcls: library ABI %d, binding ABI %d", int(v), int(C.clsg_abi_version()))
	}
	if len(devices) == 0 {
		return nil, errors.New("contivcls: no device")
	}
	var e *C.cls_engine
	dl := make([]C.int, len(devices)) // pointer-free Go memory: the shim builds cls_config
	for i, d := range devices {
		dl[i] = C.int(d)
	}
	switch rc := C.clsg_engine_create(&dl[0], C.uint32_t(len(dl)), &e); rc {
	case C.CLS_OK:
	default:
		return nil, errors.New("contivcls: no usable gfx950 device")
	}
	return &Engine{e: e, Contiv: c, pods: map[podmodel.ID]*podConfig{},
		byName: map[string]*vpp_acl.AccessLists_Acl{}}, nil
}

// Close releases the engine and its device memory.
func (en *Engine) Close() {
	en.Lock()
	defer en.Unlock()
	if en.e != nil {
		C.cls_engine_destroy(en.e)
		en.e = nil
	}
}

func (en *Engine) lastErr() error { return errors.New(C.GoString(C.cls_last_error(en.e))) }

// cstrs frees the C strings a call borrowed.
type cstrs []*C.char

func (s *cstrs) add(v string) *C.char {
	p := C.CString(v)
	*s = append(*s, p)
	return p
}

func (s cstrs) free() {
	for _, p := range s {
		C.free(unsafe.Pointer(p))
	}
}

// flatten turns the protobuf rules into cls_rule records.  Presence bits
// carry the nil-ness of every sub-message evalACL looks at
// (aclengine_mock.go:481-664); the CIDR strings go verbatim and the engine
// parses them with Go 1.9 net.ParseCIDR semantics, so unparsable strings give
// the same FAILURE verdicts.  A rule with nil Matches (a panic in evalACL) is
// rejected by cls_table_put / cls_acl_put with CLS_E_INVAL.
func flatten(acl *vpp_acl.AccessLists_Acl, strs *cstrs) []C.cls_rule {
	rules := make([]C.cls_rule, len(acl.Rules))
	for i, r := range acl.Rules {
		c := &rules[i]
		if r.Actions != nil {
			c.flags |= C.CLS_R_ACTIONS
			c.acl_action = C.int32_t(r.Actions.AclAction)
		}
		m := r.Matches
		if m == nil {
			continue
		}
		c.flags |= C.CLS_R_MATCHES
		if m.MacipRule != nil {
			c.flags |= C.CLS_R_MACIP
		}
		ip := m.IpRule
		if ip == nil {
			continue
		}
		c.flags |= C.CLS_R_IPRULE
		if ip.Ip != nil {
			c.flags |= C.CLS_R_IP
			c.src_network = strs.add(ip.Ip.SourceNetwork)
			c.dst_network = strs.add(ip.Ip.DestinationNetwork)
		}
		if ip.Other != nil {
			c.flags |= C.CLS_R_OTHER
		}
		if t := ip.Tcp; t != nil {
			c.flags |= C.CLS_R_TCP
			if p := t.SourcePortRange; p != nil {
				c.flags |= C.CLS_R_TCP_SRC
				c.tcp_src_lo, c.tcp_src_hi = C.uint32_t(p.LowerPort), C.uint32_t(p.UpperPort)
			}
			if p := t.DestinationPortRange; p != nil {
				c.flags |= C.CLS_R_TCP_DST
				c.tcp_dst_lo, c.tcp_dst_hi = C.uint32_t(p.LowerPort), C.uint32_t(p.UpperPort)
			}
		}
		if u := ip.Udp; u != nil {
			c.flags |= C.CLS_R_UDP
			if p := u.SourcePortRange; p != nil {
				c.flags |= C.CLS_R_UDP_SRC
				c.udp_src_lo, c.udp_src_hi = C.uint32_t(p.LowerPort), C.uint32_t(p.UpperPort)
			}
			if p := u.DestinationPortRange; p != nil {
				c.flags |= C.CLS_R_UDP_DST
				c.udp_dst_lo, c.udp_dst_hi = C.uint32_t(p.LowerPort), C.uint32_t(p.UpperPort)
			}
		}
		if ic := ip.Icmp; ic != nil {
			c.flags |= C.CLS_R_ICMP
			if ic.Icmpv6 {
				c.flags |= C.CLS_R_ICMPV6
			}
			if p := ic.IcmpCodeRange; p != nil {
				c.flags |= C.CLS_R_ICMP_CODE
				c.icmp_code_first, c.icmp_code_last = C.uint32_t(p.First), C.uint32_t(p.Last)
			}
			if p := ic.IcmpTypeRange; p != nil {
				c.flags |= C.CLS_R_ICMP_TYPE
				c.icmp_type_first, c.icmp_type_last = C.uint32_t(p.First), C.uint32_t(p.Last)
			}
		}
	}
	return rules
}

// RegisterPod replaces MockACLEngine.RegisterPod (aclengine_mock.go:144-148).
func (en *Engine) RegisterPod(pod podmodel.ID, podIP string, anotherNode bool) {
	en.Lock()
	defer en.Unlock()
	en.pods[pod] = &podConfig{ip: net.ParseIP(podIP), anotherNode: anotherNode}
}

// ApplyTxn replaces MockACLEngine.ApplyTxn (aclengine_mock.go:151-198): the
// engine is the onCommit of the txn tracker (mock/localclient/txn.go:120-131).
// Like the reference, an error aborts mid-transaction with no rollback.
func (en *Engine) ApplyTxn(txn *localclient.Txn) error {
	en.Lock()
	defer en.Unlock()
	if txn == nil {
		return errors.New("txn is nil")
	}
	if txn.DefaultPluginsDataChangeTxn != nil || txn.DefaultPluginsDataResyncTxn != nil {
		return errors.New("defaultplugins txn is not supported")
	}
	if txn.LinuxDataResyncTxn != nil {
		return errors.New("linux resync txn is not supported")
	}
	if txn.LinuxDataChangeTxn == nil {
		return errors.New("linux data change txn is nil")
	}
	for _, op := range txn.LinuxDataChangeTxn.Ops {
		if !strings.HasPrefix(op.Key, vpp_acl.KeyPrefix()) {
			return errors.New("non-ACL changed in txn")
		}
		if op.Value == nil {
			name := strings.TrimPrefix(op.Key, vpp_acl.KeyPrefix())
			if err := en.delACL(name); err != nil {
				return err
			}
			continue
		}
		acl, ok := op.Value.(*vpp_acl.AccessLists_Acl)
		if !ok {
			return errors.New("failed to cast ACL value")
		}
		if err := en.putACL(acl); err != nil {
			return err
		}
	}
	return nil
}

// putACL: ACLConfig.PutACL (aclengine_mock.go:699-728) in the C engine
// (empty Interfaces is an error there too; a re-put of equal rules keeps the
// compiled table and only moves the bindings).
func (en *Engine) putACL(acl *vpp_acl.AccessLists_Acl) error {
	var strs cstrs
	defer strs.free()
	rules := flatten(acl, &strs)
	var ing, eg []*C.char
	if acl.Interfaces != nil {
		for _, s := range acl.Interfaces.Ingress {
			ing = append(ing, strs.add(s))
		}
		for _, s := range acl.Interfaces.Egress {
			eg = append(eg, strs.add(s))
		}
	}
	var rp *C.cls_rule
	if len(rules) > 0 {
		rp = &rules[0]
	}
	var ip, ep **C.char
	if len(ing) > 0 {
		ip = &ing[0]
	}
	if len(eg) > 0 {
		ep = &eg[0]
	}
	if rc := C.cls_acl_put(en.e, strs.add(acl.AclName), rp, C.uint32_t(len(rules)), ip, C.uint32_t(len(ing)),
		ep, C.uint32_t(len(eg))); rc != C.CLS_OK {
		return en.lastErr()
	}
	en.byName[acl.AclName] = acl
	return nil
}

// delACL: ACLConfig.DelACL (aclengine_mock.go:680-696).
func (en *Engine) delACL(name string) error {
	var strs cstrs
	defer strs.free()
	if rc := C.cls_acl_del(en.e, strs.add(name)); rc != C.CLS_OK {
		return en.lastErr()
	}
	delete(en.byName, name)
	return nil
}

// DumpACLs replaces MockACLEngine.DumpACLs (aclengine_mock.go:201-206).
func (en *Engine) DumpACLs() (acls []*vpp_acl.AccessLists_Acl) {
	en.Lock()
	defer en.Unlock()
	for _, acl := range en.byName {
		acls = append(acls, acl)
	}
	return acls
}

// GetNumOfACLs replaces MockACLEngine.GetNumOfACLs (:209-212).
func (en *Engine) GetNumOfACLs() int {
	n, _ := en.counts()
	return n
}

// GetNumOfACLChanges replaces MockACLEngine.GetNumOfACLChanges (:237-240).
func (en *Engine) GetNumOfACLChanges() int {
	_, c := en.counts()
	return c
}

func (en *Engine) counts() (int, int) {
	en.Lock()
	defer en.Unlock()
	var n, c C.uint32_t
	C.cls_acl_counts(en.e, &n, &c)
	return int(n), int(c)
}

// aclOfTable: the installed protobuf whose compiled table the engine bound.
func (en *Engine) aclOfTable(tid C.int32_t) *vpp_acl.AccessLists_Acl {
	if tid < 0 {
		return nil
	}
	var strs cstrs
	defer strs.free()
	for name, acl := range en.byName {
		var id C.uint32_t
		if C.cls_acl_table(en.e, strs.add(name), &id) == C.CLS_OK && C.int32_t(id) == tid {
			return acl
		}
	}
	return nil
}

func (en *Engine) ifACLs(ifName string) (in, out C.int32_t) {
	var strs cstrs
	defer strs.free()
	var id C.uint32_t
	in, out = -1, -1
	if C.cls_if_id(en.e, strs.add(ifName), &id) == C.CLS_OK {
		C.cls_if_acls(en.e, id, &in, &out)
	}
	return in, out
}

// GetInboundACL replaces MockACLEngine.GetInboundACL (:215-219).
func (en *Engine) GetInboundACL(ifName string) *vpp_acl.AccessLists_Acl {
	en.Lock()
	defer en.Unlock()
	in, _ := en.ifACLs(ifName)
	return en.aclOfTable(in)
}

// GetOutboundACL replaces MockACLEngine.GetOutboundACL (:222-226).
func (en *Engine) GetOutboundACL(ifName string) *vpp_acl.AccessLists_Acl {
	en.Lock()
	defer en.Unlock()
	_, out := en.ifACLs(ifName)
	return en.aclOfTable(out)
}

// GetACLByName replaces MockACLEngine.GetACLByName (:228-234).
func (en *Engine) GetACLByName(aclName string) *vpp_acl.AccessLists_Acl {
	en.Lock()
	defer en.Unlock()
	return en.byName[aclName]
}

// Conn is one Connection* call for ConnectionBatch.  Kind selects the
// reference entry point; the fields it does not use are ignored.
type Conn struct {
	Kind           ConnKind
	SrcPod, DstPod podmodel.ID
	SrcIP, DstIP   string // ConnectionInternetToPod / ConnectionPodToInternet
	Protocol       aclengine.ProtocolType
	SrcPort        uint16
	DstPort        uint16
}

// ConnKind names the reference entry point of a Conn.
type ConnKind int

const (
	PodToPod      ConnKind = iota // ConnectionPodToPod (aclengine_mock.go:243-300)
	PodToInternet                 // ConnectionPodToInternet (:304-345)
	InternetToPod                 // ConnectionInternetToPod (:349-390)
)

// nodeOutputIf: the VXLAN BVI, else the main physical interface (:272-279).
func (en *Engine) nodeOutputIf() string {
	if ifName := en.Contiv.GetVxlanBVIIfName(); ifName != "" {
		return ifName
	}
	return en.Contiv.GetMainPhysicalIfName()
}

func (en *Engine) podIf(pod podmodel.ID, cfg *podConfig) (string, bool) {
	if cfg.anotherNode {
		ifName := en.nodeOutputIf()
		return ifName, ifName != ""
	}
	return en.Contiv.GetIfName(pod.Namespace, pod.Name)
}

// resolve: interfaces and addresses of a call, as the reference finds them
// before testConnection; ok == false is ConnActionFailure.
func (en *Engine) resolve(c *Conn) (srcIf, dstIf string, srcIP, dstIP net.IP, ok bool) {
	switch c.Kind {
	case PodToPod:
		s, d := en.pods[c.SrcPod], en.pods[c.DstPod]
		if s == nil || d == nil {
			return
		}
		var ok1, ok2 bool
		srcIf, ok1 = en.podIf(c.SrcPod, s)
		dstIf, ok2 = en.podIf(c.DstPod, d)
		return srcIf, dstIf, s.ip, d.ip, ok1 && ok2
	case PodToInternet:
		s := en.pods[c.SrcPod]
		if s == nil || s.anotherNode {
			return
		}
		var ok1 bool
		srcIf, ok1 = en.Contiv.GetIfName(c.SrcPod.Namespace, c.SrcPod.Name)
		dstIf, dstIP = en.nodeOutputIf(), net.ParseIP(c.DstIP)
		return srcIf, dstIf, s.ip, dstIP, ok1 && dstIf != "" && dstIP != nil
	default:
		d := en.pods[c.DstPod]
		if d == nil || d.anotherNode {
			return
		}
		var ok2 bool
		srcIf, srcIP = en.nodeOutputIf(), net.ParseIP(c.SrcIP)
		dstIf, ok2 = en.Contiv.GetIfName(c.DstPod.Namespace, c.DstPod.Name)
		return srcIf, dstIf, srcIP, d.ip, srcIf != "" && srcIP != nil && ok2
	}
}

// ConnectionBatch evaluates many Connection* calls in one GPU launch
// (testConnection, aclengine_mock.go:394-471, per call): the IPv4 layout when
// every endpoint is IPv4, else the 16-byte layout (IPv4 as IPv4-mapped, as
// Go's To4).  count: add every evalACL call's terminating rule to the tables'
// connection counters (cls_conn_counters).
func (en *Engine) ConnectionBatch(calls []Conn, count bool) ([]aclengine.ConnectionAction, error) {
	en.Lock()
	defer en.Unlock()
	out := make([]aclengine.ConnectionAction, len(calls))
	var idx []int
	var sif, dif []uint32
	var sip, dip []net.IP
	var proto []uint8
	var sport, dport []uint16
	var strs cstrs
	defer strs.free()
	ifID := map[string]uint32{}
	id := func(name string) uint32 {
		if v, ok := ifID[name]; ok {
			return v
		}
		var v C.uint32_t
		C.cls_if_id(en.e, strs.add(name), &v)
		ifID[name] = uint32(v)
		return uint32(v)
	}
	v4 := true
	for i := range calls {
		s, d, a, b, ok := en.resolve(&calls[i])
		if !ok {
			out[i] = aclengine.ConnActionFailure
			continue
		}
		idx = append(idx, i)
		sif, dif = append(sif, id(s)), append(dif, id(d))
		sip, dip = append(sip, a), append(dip, b)
		proto = append(proto, uint8(calls[i].Protocol))
		sport, dport = append(sport, calls[i].SrcPort), append(dport, calls[i].DstPort)
		v4 = v4 && a.To4() != nil && b.To4() != nil
	}
	n := len(idx)
	if n == 0 {
		return out, nil
	}
	// every slice goes to the shim as its own pointer (pointer-free Go
	// memory); the shim builds cls_conn_soa on the C stack
	res := make([]uint8, n)
	flags := C.uint32_t(0)
	if count {
		flags |= C.CLS_F_COUNT
	}
	var rc C.int
	if v4 {
		s4, d4 := make([]uint32, n), make([]uint32, n)
		for k := 0; k < n; k++ {
			a, b := sip[k].To4(), dip[k].To4()
			s4[k] = uint32(a[0])<<24 | uint32(a[1])<<16 | uint32(a[2])<<8 | uint32(a[3])
			d4[k] = uint32(b[0])<<24 | uint32(b[1])<<16 | uint32(b[2])<<8 | uint32(b[3])
		}
		rc = C.clsg_connect_v4(en.e, (*C.uint32_t)(&sif[0]), (*C.uint32_t)(&dif[0]), (*C.uint32_t)(&s4[0]),
			(*C.uint32_t)(&d4[0]), (*C.uint16_t)(&sport[0]), (*C.uint16_t)(&dport[0]), (*C.uint8_t)(&proto[0]),
			C.uint64_t(n), (*C.uint8_t)(&res[0]), flags)
	} else {
		s16, d16 := make([]byte, 16*n), make([]byte, 16*n)
		for k := 0; k < n; k++ {
			a, b := sip[k].To16(), dip[k].To16()
			if a == nil || b == nil {
				return nil, errors.New("connection endpoint is not an IPv4 or IPv6 address")
			}
			copy(s16[16*k:], a)
			copy(d16[16*k:], b)
		}
		rc = C.clsg_connect_v16(en.e, (*C.uint32_t)(&sif[0]), (*C.uint32_t)(&dif[0]), (*C.uint8_t)(&s16[0]),
			(*C.uint8_t)(&d16[0]), (*C.uint16_t)(&sport[0]), (*C.uint16_t)(&dport[0]), (*C.uint8_t)(&proto[0]),
			C.uint64_t(n), (*C.uint8_t)(&res[0]), flags)
	}
	if rc != C.CLS_OK {
		return nil, en.lastErr()
	}
	for k, i := range idx {
		out[i] = aclengine.ConnectionAction(res[k])
	}
	return out, nil
}

// ConnectionPodToPod replaces MockACLEngine.ConnectionPodToPod (:243-300).
func (en *Engine) ConnectionPodToPod(srcPod podmodel.ID, dstPod podmodel.ID, protocol aclengine.ProtocolType,
	srcPort uint16, dstPort uint16) aclengine.ConnectionAction {
	return en.one(Conn{Kind: PodToPod, SrcPod: srcPod, DstPod: dstPod, Protocol: protocol,
		SrcPort: srcPort, DstPort: dstPort})
}

// ConnectionPodToInternet replaces MockACLEngine.ConnectionPodToInternet (:304-345).
func (en *Engine) ConnectionPodToInternet(srcPod podmodel.ID, dstIP string, protocol aclengine.ProtocolType,
	srcPort uint16, dstPort uint16) aclengine.ConnectionAction {
	return en.one(Conn{Kind: PodToInternet, SrcPod: srcPod, DstIP: dstIP, Protocol: protocol,
		SrcPort: srcPort, DstPort: dstPort})
}

// ConnectionInternetToPod replaces MockACLEngine.ConnectionInternetToPod (:349-390).
func (en *Engine) ConnectionInternetToPod(srcIP string, dstPod podmodel.ID, protocol aclengine.ProtocolType,
	srcPort uint16, dstPort uint16) aclengine.ConnectionAction {
	return en.one(Conn{Kind: InternetToPod, SrcIP: srcIP, DstPod: dstPod, Protocol: protocol,
		SrcPort: srcPort, DstPort: dstPort})
}

func (en *Engine) one(c Conn) aclengine.ConnectionAction {
	res, err := en.ConnectionBatch([]Conn{c}, false)
	if err != nil {
		return aclengine.ConnActionFailure
	}
	return res[0]
}

// Table is one compiled ACL on the device (cls_table_put), for batched
// classification outside the renderer's bindings.
type Table struct {
	ID     uint32
	NRules int
}

// PutTable compiles and uploads an ACL's rules (evalACL semantics).
func (en *Engine) PutTable(acl *vpp_acl.AccessLists_Acl) (*Table, error) {
	en.Lock()
	defer en.Unlock()
	var strs cstrs
	defer strs.free()
	rules := flatten(acl, &strs)
	var rp *C.cls_rule
	if len(rules) > 0 {
		rp = &rules[0]
	}
	var id C.uint32_t
	if rc := C.cls_table_put(en.e, strs.add(acl.AclName), rp, C.uint32_t(len(rules)), &id); rc != C.CLS_OK {
		return nil, en.lastErr()
	}
	return &Table{ID: uint32(id), NRules: len(rules)}, nil
}

// DelTable frees a table (its pending device work finishes first).
func (en *Engine) DelTable(t *Table) error {
	en.Lock()
	defer en.Unlock()
	if rc := C.cls_table_del(en.e, C.uint32_t(t.ID)); rc != C.CLS_OK {
		return en.lastErr()
	}
	return nil
}

// ClassifyBatch: evalACL (aclengine_mock.go:473-668) for every packet of an
// IPv4 batch (host-order addresses), and the per-rule hit counters
// (counters[k], k < R: packets that terminated at rule k; counters[R]: the
// default DENY).
func (en *Engine) ClassifyBatch(t *Table, src, dst []uint32, dport []uint16,
	proto []aclengine.ProtocolType) ([]uint8, []uint64, error) {
	n := len(src)
	if len(dst) != n || len(dport) != n || len(proto) != n {
		return nil, nil, errors.New("contivcls: packet arrays of different lengths")
	}
	verdict := make([]uint8, n)
	counters := make([]uint64, t.NRules+1)
	if n == 0 {
		return verdict, counters, nil
	}
	pr := make([]uint8, n)
	for i, p := range proto {
		pr[i] = uint8(p)
	}
	en.Lock()
	defer en.Unlock()
	if rc := C.clsg_classify_v4(en.e, C.uint32_t(t.ID), (*C.uint32_t)(&src[0]), (*C.uint32_t)(&dst[0]),
		(*C.uint16_t)(&dport[0]), (*C.uint8_t)(&pr[0]), C.uint64_t(n), (*C.uint8_t)(&verdict[0]),
		(*C.uint64_t)(&counters[0]), 0); rc != C.CLS_OK {
		return nil, nil, en.lastErr()
	}
	return verdict, counters, nil
}

// ClassifyBatchRules: each packet's ACLAction and the index of the rule at
// which evalACL terminated (t.NRules: the default DENY) -- the matched rule
// evalACL logs at Debug (aclengine_mock.go:651-654), for a whole batch; no
// counters.
func (en *Engine) ClassifyBatchRules(t *Table, src, dst []uint32, dport []uint16,
	proto []aclengine.ProtocolType) ([]uint8, []uint32, error) {
	n := len(src)
	if len(dst) != n || len(dport) != n || len(proto) != n {
		return nil, nil, errors.New("contivcls: packet arrays of different lengths")
	}
	verdict := make([]uint8, n)
	rules := make([]uint32, n)
	if n == 0 {
		return verdict, rules, nil
	}
	pr := make([]uint8, n)
	for i, p := range proto {
		pr[i] = uint8(p)
	}
	en.Lock()
	defer en.Unlock()
	if rc := C.clsg_classify_rules_v4(en.e, C.uint32_t(t.ID), (*C.uint32_t)(&src[0]), (*C.uint32_t)(&dst[0]),
		(*C.uint16_t)(&dport[0]), (*C.uint8_t)(&pr[0]), C.uint64_t(n), (*C.uint8_t)(&verdict[0]),
		(*C.uint32_t)(&rules[0])); rc != C.CLS_OK {
		return nil, nil, en.lastErr()
	}
	return verdict, rules, nil
}

// ClassifyBatchIP: the same for addresses of any family (net.IP; IPv4 and
// IPv4-mapped packets match IPv4 networks only, as Go's IPNet.Contains).
func (en *Engine) ClassifyBatchIP(t *Table, src, dst []net.IP, dport []uint16,
	proto []aclengine.ProtocolType) ([]uint8, []uint64, error) {
	n := len(src)
	if len(dst) != n || len(dport) != n || len(proto) != n {
		return nil, nil, errors.New("contivcls: packet arrays of different lengths")
	}
	verdict := make([]uint8, n)
	counters := make([]uint64, t.NRules+1)
	if n == 0 {
		return verdict, counters, nil
	}
	s16, d16, pr := make([]byte, 16*n), make([]byte, 16*n), make([]uint8, n)
	for i := 0; i < n; i++ {
		a, b := src[i].To16(), dst[i].To16()
		if a == nil || b == nil {
			return nil, nil, errors.New("contivcls: packet address is not an IPv4 or IPv6 address")
		}
		copy(s16[16*i:], a)
		copy(d16[16*i:], b)
		pr[i] = uint8(proto[i])
	}
	en.Lock()
	defer en.Unlock()
	if rc := C.clsg_classify_v16(en.e, C.uint32_t(t.ID), (*C.uint8_t)(&s16[0]), (*C.uint8_t)(&d16[0]),
		(*C.uint16_t)(&dport[0]), (*C.uint8_t)(&pr[0]), C.uint64_t(n), (*C.uint8_t)(&verdict[0]),
		(*C.uint64_t)(&counters[0]), 0); rc != C.CLS_OK {
		return nil, nil, en.lastErr()
	}
	return verdict, counters, nil
}

// ConnCounters: the per-(ACL, rule) hit counters of the connection path for
// the installed ACL aclName (cls_conn_counters; reset clears them).
func (en *Engine) ConnCounters(aclName string, reset bool) ([]uint64, error) {
	en.Lock()
	defer en.Unlock()
	var strs cstrs
	defer strs.free()
	var id C.uint32_t
	if rc := C.cls_acl_table(en.e, strs.add(aclName), &id); rc != C.CLS_OK {
		return nil, en.lastErr()
	}
	var info C.cls_table_info
	if rc := C.cls_table_get_info(en.e, id, &info); rc != C.CLS_OK {
		return nil, en.lastErr()
	}
	out := make([]uint64, int(info.n_rules)+1)
	r := C.uint32_t(0)
	if reset {
		r = 1
	}
	if rc := C.cls_conn_counters(en.e, id, (*C.uint64_t)(&out[0]), r); rc != C.CLS_OK {
		return nil, en.lastErr()
	}
	return out, nil
}

// ---- HBM-resident batches (ABI 4) -------------------------------------------
// A Batch is engine-owned memory: packets stay in HBM between calls and no
// Go pointer is ever kept by the library (cgo rule).  With mirror the batch
// also owns pinned host arrays (Mirror*) that Go fills in place; Upload(f,
// nil) then moves them at DMA speed.

// Batch fields (CLS_BF_*).
const (
	FieldSrc     = uint32(C.CLS_BF_SRC)
	FieldDst     = uint32(C.CLS_BF_DST)
	FieldSport   = uint32(C.CLS_BF_SPORT)
	FieldDport   = uint32(C.CLS_BF_DPORT)
	FieldProto   = uint32(C.CLS_BF_PROTO)
	FieldVerdict = uint32(C.CLS_BF_VERDICT)
	FieldSrcIf   = uint32(C.CLS_BF_SRC_IF)
	FieldDstIf   = uint32(C.CLS_BF_DST_IF)
)

type Batch struct {
	en *Engine
	b  *C.cls_batch
	N  int
	V6 bool
}

// NewBatch: n IPv4 (v6 false: host-order u32 addresses) or 16-byte packets;
// conn adds interface ids (ConnectBatchDevice).
func (en *Engine) NewBatch(n int, v6, conn, mirror bool) (*Batch, error) {
	en.Lock()
	defer en.Unlock()
	af := C.uint32_t(C.CLS_AF_V4)
	if v6 {
		af = C.CLS_AF_V16
	}
	fl := C.uint32_t(0)
	if conn {
		fl |= C.CLS_BATCH_CONN
	}
	if mirror {
		fl |= C.CLS_BATCH_MIRROR
	}
	var b *C.cls_batch
	if rc := C.cls_batch_create(en.e, af, C.uint64_t(n), fl, &b); rc != C.CLS_OK {
		return nil, en.lastErr()
	}
	return &Batch{en: en, b: b, N: n, V6: v6}, nil
}

// Close frees the batch (before its engine).
func (b *Batch) Close() {
	if b.b != nil {
		C.cls_batch_destroy(b.b)
		b.b = nil
	}
}

// MirrorU32 / MirrorU16 / MirrorU8: the pinned host array of a field (C
// memory: Go may keep and fill these slices), nil without CLS_BATCH_MIRROR.
// Go 1.9 slices C memory through a large array type (no unsafe.Slice).
func (b *Batch) MirrorU32(f uint32) []uint32 {
	p := C.clsg_batch_mirror(b.b, C.uint32_t(f))
	if p == nil {
		return nil
	}
	return (*[1 << 32]uint32)(p)[:b.N:b.N]
}
func (b *Batch) MirrorU16(f uint32) []uint16 {
	p := C.clsg_batch_mirror(b.b, C.uint32_t(f))
	if p == nil {
		return nil
	}
	return (*[1 << 33]uint16)(p)[:b.N:b.N]
}
func (b *Batch) MirrorU8(f uint32) []uint8 {
	p := C.clsg_batch_mirror(b.b, C.uint32_t(f))
	if p == nil {
		return nil
	}
	return (*[1 << 34]uint8)(p)[:b.N:b.N]
}

// Upload packets [first, first+n) of a field from src (the base of a Go
// slice of the field's element type: pointer-free Go memory, valid for the
// call), or from the mirror (src nil).
func (b *Batch) Upload(f uint32, first, n int, src unsafe.Pointer) error {
	if rc := C.cls_batch_upload(b.b, C.uint32_t(f), C.uint64_t(first), C.uint64_t(n), src); rc != C.CLS_OK {
		return b.en.lastErr()
	}
	return nil
}

// Verdicts of packets [first, first+n) (waits for the batch's work).
func (b *Batch) Verdicts(first, n int) ([]uint8, error) {
	out := make([]uint8, n)
	if n == 0 {
		return out, nil
	}
	if rc := C.cls_batch_download(b.b, C.CLS_BF_VERDICT, C.uint64_t(first), C.uint64_t(n),
		unsafe.Pointer(&out[0])); rc != C.CLS_OK {
		return nil, b.en.lastErr()
	}
	return out, nil
}

// ClassifyBatchDevice: evalACL over the whole batch on its devices; the hit
// counters summed over the shards (and over processes, CommInit).  wait
// false only enqueues (Counters reads the last call's).
func (en *Engine) ClassifyBatchDevice(t *Table, b *Batch, wait bool) ([]uint64, error) {
	var out []uint64
	var op *C.uint64_t
	if wait {
		out = make([]uint64, t.NRules+1)
		op = (*C.uint64_t)(&out[0])
	}
	if rc := C.cls_classify_batch(en.e, C.uint32_t(t.ID), b.b, op, 0); rc != C.CLS_OK {
		return nil, en.lastErr()
	}
	return out, nil
}

// Counters of the batch's last ClassifyBatchDevice.
func (b *Batch) Counters(t *Table) ([]uint64, error) {
	out := make([]uint64, t.NRules+1)
	if rc := C.cls_batch_counters(b.b, (*C.uint64_t)(&out[0]), C.uint32_t(len(out))); rc != C.CLS_OK {
		return nil, b.en.lastErr()
	}
	return out, nil
}

// ConnectBatchDevice: testConnection over a conn batch (ConnectionAction per
// connection into FieldVerdict).
func (en *Engine) ConnectBatchDevice(b *Batch, count bool) error {
	fl := C.uint32_t(0)
	if count {
		fl |= C.CLS_F_COUNT
	}
	if rc := C.cls_batch_connect(en.e, b.b, fl); rc != C.CLS_OK {
		return en.lastErr()
	}
	return nil
}

// CommUniqueID / CommInit: one process per GPU (or GPU group) joins one RCCL
// communicator for the counter merge; process 0 makes the id, the others get
// it out of band.
func CommUniqueID() ([128]byte, error) {
	var id [128]byte
	if rc := C.cls_comm_unique_id(unsafe.Pointer(&id[0])); rc != C.CLS_OK {
		return id, errors.New("contivcls: RCCL unavailable")
	}
	return id, nil
}

func (en *Engine) CommInit(nProcs, proc int, id *[128]byte) error {
	var p unsafe.Pointer
	if id != nil {
		p = C.CBytes(id[:])
		defer C.free(p)
	}
	if rc := C.cls_comm_init(en.e, C.uint32_t(nProcs), C.uint32_t(proc), p); rc != C.CLS_OK {
		return en.lastErr()
	}
	return nil
}
