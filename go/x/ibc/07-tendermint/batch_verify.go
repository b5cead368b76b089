package tendermint

// Batched commit-signature checks for the IBC 07-tendermint light client
// (SURVEY.md §8f-4).  The reference checks a header in checkValidity
// (x/ibc/07-tendermint/update.go:88: lite.Verify -> VerifyAdjacent /
// VerifyNonAdjacent) and misbehaviour in checkMisbehaviour
// (misbehaviour.go:88-97: two VerifyCommitTrusting calls); every validator
// signature goes through PubKeyEd25519.VerifyBytes one at a time inside
// tendermint v0.33.4 types/validator_set.go VerifyCommit /
// VerifyCommitTrusting.  Here every signature those loops could read is
// verified in ONE gpuverify.EdVerifier batch (gv_verify_ed25519_msgs), and the
// loops then run in reference order over the verdicts: the same first wrong
// signature, the same tallies, the same early return, the same errors.
//
// Wiring (two call sites, INTEGRATION.md):
//   update.go:88        lite.Verify(...)                   -> BatchVerify(commitVerifier, ...)
//   misbehaviour.go:88  two ValidatorSet.VerifyCommitTrusting -> VerifyCommits(commitVerifier, both)
// SetCommitVerifier installs the verifier at app construction; nil keeps the
// reference's CPU path (gpuverify.CPU).
//
// Source-level only here (no Go toolchain in the build image); the C++
// mirror gvh_verify_commits (host/gvhost.cpp) implements the same loops and
// is tested against a sequential restatement (tests/test_ibc_commits.py).

import (
	"bytes"
	"fmt"
	"time"

	"github.com/pkg/errors"
	"github.com/tendermint/tendermint/crypto/ed25519"
	tmmath "github.com/tendermint/tendermint/libs/math"
	lite "github.com/tendermint/tendermint/lite2"
	tmtypes "github.com/tendermint/tendermint/types"

	gv "github.com/cosmos/cosmos-sdk/crypto/gpuverify"
)

var commitVerifier gv.EdVerifier = gv.CPU{}

// SetCommitVerifier routes the light client's commit signatures to ev (a
// *gpuverify.GPU); nil restores the CPU path.
func SetCommitVerifier(ev gv.EdVerifier) {
	if ev == nil {
		ev = gv.CPU{}
	}
	commitVerifier = ev
}

// CommitCheck is one VerifyCommit (Trusting == false) or VerifyCommitTrusting
// call: the arguments of the reference method, receiver first.
type CommitCheck struct {
	Vals       *tmtypes.ValidatorSet
	ChainID    string
	BlockID    tmtypes.BlockID
	Height     int64
	Commit     *tmtypes.Commit
	Trusting   bool
	TrustLevel tmmath.Fraction
	// KeysTrusted: Vals is a set the client already trusts (the trusted
	// next-validator set of VerifyCommitTrusting, or an adjacent header's set
	// whose hash equals the trusted header's NextValidatorsHash).  Only such
	// sets' keys go through the resident-key path (gv.EdKeyCache): a set
	// supplied by an arbitrary relayer is verified without loading its keys,
	// so fresh keys in every MsgUpdateClient cannot churn the key arena and
	// evict the honest sets it keeps.
	KeysTrusted bool
}

// leaf: one signature a check's loop could read, and its batch position.
type leaf struct {
	val   int // validator index in the check's set
	item  int // batch item, -1: VerifyBytes is false without verifying (len(sig) != 64)
	plain bool // item indexes the plain (untrusted keys) batch
}

// edBatch gathers one verification batch.
type edBatch struct {
	pubs       []ed25519.PubKeyEd25519
	msgs, sigs [][]byte
	ok         []bool
}

func (b *edBatch) add(pk ed25519.PubKeyEd25519, msg, sig []byte) int {
	b.pubs = append(b.pubs, pk)
	b.msgs = append(b.msgs, msg)
	b.sigs = append(b.sigs, sig)
	return len(b.pubs) - 1
}

// VerifyCommits returns, for each check, exactly the error the reference
// method returns (nil on success), with the signatures of all checks
// verified in one batch.  The trust-level sanity check panics like the
// reference (validator_set.go VerifyCommitTrusting).
func VerifyCommits(ev gv.EdVerifier, checks []CommitCheck) []error {
	errs := make([]error, len(checks))
	leaves := make([][]leaf, len(checks))
	var cached, plain edBatch // trusted sets' keys may stay resident; untrusted sets' are not loaded
	for c, k := range checks {
		if k.Trusting {
			if k.TrustLevel.Numerator*3 < k.TrustLevel.Denominator || // < 1/3
				k.TrustLevel.Numerator > k.TrustLevel.Denominator { // > 1
				panic(fmt.Sprintf("trustLevel must be within [1/3, 1], given %v", k.TrustLevel))
			}
		} else if k.Vals.Size() != len(k.Commit.Signatures) {
			errs[c] = tmtypes.NewErrInvalidCommitSignatures(k.Vals.Size(), len(k.Commit.Signatures))
			continue
		}
		if err := verifyCommitBasic(k.Commit, k.Height, k.BlockID); err != nil {
			errs[c] = err
			continue
		}
		lv := make([]leaf, len(k.Commit.Signatures))
		for idx, cs := range k.Commit.Signatures {
			lv[idx] = leaf{val: -1, item: -1}
			if cs.Absent() {
				continue
			}
			v := idx // VerifyCommit: the vals and commit correspond 1:1
			if k.Trusting {
				v, _ = k.Vals.GetByAddress(cs.ValidatorAddress)
			}
			lv[idx].val = v
			if v < 0 {
				continue
			}
			pk, ok := k.Vals.Validators[v].PubKey.(ed25519.PubKeyEd25519)
			if !ok || len(cs.Signature) != ed25519.SignatureSize {
				continue // resolved one at a time below (non-ed25519 key) or false (length)
			}
			msg := k.Commit.VoteSignBytes(k.ChainID, idx)
			if k.KeysTrusted {
				lv[idx].item = cached.add(pk, msg, cs.Signature)
			} else {
				lv[idx].item, lv[idx].plain = plain.add(pk, msg, cs.Signature), true
			}
		}
		leaves[c] = lv
	}
	if len(cached.pubs) > 0 {
		if kc, isCache := ev.(gv.EdKeyCache); isCache {
			cached.ok = kc.VerifyBatchEd25519Cached(cached.pubs, cached.msgs, cached.sigs) // trusted sets repeat
		} else {
			cached.ok = ev.VerifyBatchEd25519(cached.pubs, cached.msgs, cached.sigs)
		}
	}
	if len(plain.pubs) > 0 {
		plain.ok = ev.VerifyBatchEd25519(plain.pubs, plain.msgs, plain.sigs)
	}
	verdict := func(k CommitCheck, lf leaf, idx int) bool {
		if lf.item >= 0 {
			if lf.plain {
				return plain.ok[lf.item]
			}
			return cached.ok[lf.item]
		}
		cs := k.Commit.Signatures[idx]
		if _, isEd := k.Vals.Validators[lf.val].PubKey.(ed25519.PubKeyEd25519); isEd {
			return false // a 64-byte length check failed
		}
		return k.Vals.Validators[lf.val].PubKey.VerifyBytes(k.Commit.VoteSignBytes(k.ChainID, idx), cs.Signature)
	}
	for c, k := range checks {
		if errs[c] != nil || leaves[c] == nil {
			continue
		}
		if k.Trusting {
			errs[c] = walkTrusting(k, leaves[c], verdict)
		} else {
			errs[c] = walkCommit(k, leaves[c], verdict)
		}
	}
	return errs
}

// walkCommit is VerifyCommit's loop (validator_set.go) over batch verdicts.
func walkCommit(k CommitCheck, lv []leaf, verdict func(CommitCheck, leaf, int) bool) error {
	talliedVotingPower := int64(0)
	votingPowerNeeded := k.Vals.TotalVotingPower() * 2 / 3
	for idx, cs := range k.Commit.Signatures {
		if cs.Absent() {
			continue // OK, some signatures can be absent.
		}
		if !verdict(k, lv[idx], idx) {
			return fmt.Errorf("wrong signature (#%d): %X", idx, cs.Signature)
		}
		if k.BlockID.Equals(cs.BlockID(k.Commit.BlockID)) {
			talliedVotingPower += k.Vals.Validators[idx].VotingPower
		}
	}
	if got, needed := talliedVotingPower, votingPowerNeeded; got <= needed {
		return tmtypes.ErrNotEnoughVotingPowerSigned{Got: got, Needed: needed}
	}
	return nil
}

// walkTrusting is VerifyCommitTrusting's loop (validator_set.go) over batch
// verdicts: lookups by address, double votes, early return.
func walkTrusting(k CommitCheck, lv []leaf, verdict func(CommitCheck, leaf, int) bool) error {
	var (
		talliedVotingPower int64
		seenVals           = make(map[int]int, len(k.Commit.Signatures)) // validator index -> commit index
		votingPowerNeeded  = (k.Vals.TotalVotingPower() * k.TrustLevel.Numerator) / k.TrustLevel.Denominator
	)
	for idx, cs := range k.Commit.Signatures {
		if cs.Absent() {
			continue // OK, some signatures can be absent.
		}
		valIdx := lv[idx].val
		if firstIndex, ok := seenVals[valIdx]; ok { // double vote
			secondIndex := idx
			_, val := k.Vals.GetByAddress(cs.ValidatorAddress)
			return errors.Errorf("double vote from %v (%d and %d)", val, firstIndex, secondIndex)
		}
		if valIdx >= 0 {
			seenVals[valIdx] = idx
			if !verdict(k, lv[idx], idx) {
				return errors.Errorf("wrong signature (#%d): %X", idx, cs.Signature)
			}
			if k.BlockID.Equals(cs.BlockID(k.Commit.BlockID)) {
				talliedVotingPower += k.Vals.Validators[valIdx].VotingPower
			}
			if talliedVotingPower > votingPowerNeeded {
				return nil
			}
		}
	}
	return tmtypes.ErrNotEnoughVotingPowerSigned{Got: talliedVotingPower, Needed: votingPowerNeeded}
}

// verifyCommitBasic restates validator_set.go's unexported helper.
func verifyCommitBasic(commit *tmtypes.Commit, height int64, blockID tmtypes.BlockID) error {
	if err := commit.ValidateBasic(); err != nil {
		return err
	}
	if height != commit.Height {
		return tmtypes.NewErrInvalidCommitHeight(height, commit.Height)
	}
	if !blockID.Equals(commit.BlockID) {
		return fmt.Errorf("invalid commit -- wrong block ID: want %v, got %v", blockID, commit.BlockID)
	}
	return nil
}

// BatchVerify is lite2.Verify (tendermint v0.33.4 lite2/verifier.go) with its
// commit checks through VerifyCommits: VerifyNonAdjacent's two checks (the
// trusted set's VerifyCommitTrusting, then the new set's VerifyCommit) share
// one batch; their order of precedence is the reference's.
func BatchVerify(ev gv.EdVerifier, chainID string, trustedHeader *tmtypes.SignedHeader,
	trustedNextVals *tmtypes.ValidatorSet, untrustedHeader *tmtypes.SignedHeader,
	untrustedVals *tmtypes.ValidatorSet, trustingPeriod time.Duration, now time.Time,
	maxClockDrift time.Duration, trustLevel tmmath.Fraction) error {

	adjacent := untrustedHeader.Height == trustedHeader.Height+1
	if lite.HeaderExpired(trustedHeader, trustingPeriod, now) {
		return lite.ErrOldHeaderExpired{At: trustedHeader.Time.Add(trustingPeriod), Now: now}
	}
	if err := verifyNewHeaderAndVals(chainID, untrustedHeader, untrustedVals, trustedHeader, now, maxClockDrift); err != nil {
		return lite.ErrInvalidHeader{Reason: err}
	}
	full := CommitCheck{Vals: untrustedVals, ChainID: chainID, BlockID: untrustedHeader.Commit.BlockID,
		Height: untrustedHeader.Height, Commit: untrustedHeader.Commit}
	if adjacent {
		if !bytes.Equal(untrustedHeader.ValidatorsHash, trustedHeader.NextValidatorsHash) {
			return errors.Errorf("expected old header next validators (%X) to match those from new header (%X)",
				trustedHeader.NextValidatorsHash, untrustedHeader.ValidatorsHash)
		}
		// untrustedVals hashes to the trusted header's next validators (checked
		// just above and in verifyNewHeaderAndVals): a trusted set
		full.KeysTrusted = true
		if err := VerifyCommits(ev, []CommitCheck{full})[0]; err != nil {
			return lite.ErrInvalidHeader{Reason: err}
		}
		return nil
	}
	trusted := CommitCheck{Vals: trustedNextVals, ChainID: chainID, BlockID: untrustedHeader.Commit.BlockID,
		Height: untrustedHeader.Height, Commit: untrustedHeader.Commit, Trusting: true, TrustLevel: trustLevel,
		KeysTrusted: true}
	errs := VerifyCommits(ev, []CommitCheck{trusted, full})
	if err := errs[0]; err != nil {
		switch e := err.(type) {
		case tmtypes.ErrNotEnoughVotingPowerSigned:
			return lite.ErrNewValSetCantBeTrusted{Reason: e}
		default:
			return e
		}
	}
	if err := errs[1]; err != nil {
		return lite.ErrInvalidHeader{Reason: err}
	}
	return nil
}

// verifyNewHeaderAndVals restates lite2/verifier.go's unexported helper.
func verifyNewHeaderAndVals(chainID string, untrustedHeader *tmtypes.SignedHeader,
	untrustedVals *tmtypes.ValidatorSet, trustedHeader *tmtypes.SignedHeader, now time.Time,
	maxClockDrift time.Duration) error {

	if err := untrustedHeader.ValidateBasic(chainID); err != nil {
		return errors.Wrap(err, "untrustedHeader.ValidateBasic failed")
	}
	if untrustedHeader.Height <= trustedHeader.Height {
		return errors.Errorf("expected new header height %d to be greater than one of old header %d",
			untrustedHeader.Height, trustedHeader.Height)
	}
	if !untrustedHeader.Time.After(trustedHeader.Time) {
		return errors.Errorf("expected new header time %v to be after old header time %v",
			untrustedHeader.Time, trustedHeader.Time)
	}
	if !untrustedHeader.Time.Before(now.Add(maxClockDrift)) {
		return errors.Errorf("new header has a time from the future %v (now: %v; max clock drift: %v)",
			untrustedHeader.Time, now, maxClockDrift)
	}
	if !bytes.Equal(untrustedHeader.ValidatorsHash, untrustedVals.Hash()) {
		return errors.Errorf("expected new header validators (%X) to match those that were supplied (%X) at height %d",
			untrustedHeader.ValidatorsHash, untrustedVals.Hash(), untrustedHeader.Height)
	}
	return nil
}

// CheckMisbehaviourCommits is checkMisbehaviour's two VerifyCommitTrusting
// calls (misbehaviour.go:88-100) as one batch, with the reference's wrapping.
func CheckMisbehaviourCommits(ev gv.EdVerifier, trusted *tmtypes.ValidatorSet, chainID string,
	h1, h2 *tmtypes.SignedHeader) error {
	errs := VerifyCommits(ev, []CommitCheck{
		{Vals: trusted, ChainID: chainID, BlockID: h1.Commit.BlockID, Height: h1.Height, Commit: h1.Commit,
			Trusting: true, TrustLevel: lite.DefaultTrustLevel, KeysTrusted: true},
		{Vals: trusted, ChainID: chainID, BlockID: h2.Commit.BlockID, Height: h2.Height, Commit: h2.Commit,
			Trusting: true, TrustLevel: lite.DefaultTrustLevel, KeysTrusted: true},
	})
	if errs[0] != nil {
		return fmt.Errorf("validator set in header 1 has too much change from last known validator set: %v", errs[0])
	}
	if errs[1] != nil {
		return fmt.Errorf("validator set in header 2 has too much change from last known validator set: %v", errs[1])
	}
	return nil
}
