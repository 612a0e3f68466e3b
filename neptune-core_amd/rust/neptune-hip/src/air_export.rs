//! triton-air's constraints as the verifier's AIR descriptor (`nhip_air_create`; format: DESIGN.md
//! §9 of the neptune-hip repository).
//!
//! `triton_vm::verify` evaluates the AIR at the out-of-domain point with code that triton-vm's
//! build script generates from triton-air 1.0.0's constraint circuits (Cargo.lock:4194) through
//! triton-constraint-builder 1.0.0 (Cargo.lock:4208): `Constraints::all()`, lowered to the target
//! degree by substitution (which adds the degree-lowering columns of the master tables), then
//! combined with the substitution-induced constraints, in `init / cons / tran / term` order.  This
//! module performs the same construction and, instead of generating Rust, walks the circuits
//! (triton-constraint-circuit 1.0.0, Cargo.lock:4226) into descriptor words:
//!
//! | `CircuitExpression`                          | descriptor node                              |
//! |----------------------------------------------|----------------------------------------------|
//! | `Input(SingleRowIndicator::Main(i))`         | `INPUT` kind 0 (main, current row), index i  |
//! | `Input(SingleRowIndicator::Aux(i))`          | `INPUT` kind 1 (aux, current row), index i   |
//! | `Input(DualRowIndicator::CurrentMain(i))`    | `INPUT` kind 0, index i                      |
//! | `Input(DualRowIndicator::CurrentAux(i))`     | `INPUT` kind 1, index i                      |
//! | `Input(DualRowIndicator::NextMain(i))`       | `INPUT` kind 2 (main, next row), index i     |
//! | `Input(DualRowIndicator::NextAux(i))`        | `INPUT` kind 3 (aux, next row), index i      |
//! | `Challenge(i)`                               | `INPUT` kind 4, index i = `ChallengeId` index |
//! | `BConst(b)`                                  | `CONST` (b, 0, 0)                            |
//! | `XConst(x)`                                  | `CONST` (x0, x1, x2)                         |
//! | `BinOp(Add, a, b)`                           | `ADD` a, b                                   |
//! | `BinOp(Mul, a, b)`                           | `MUL` a, b                                   |
//!
//! Challenge indices go through unchanged: the descriptor's challenge vector is triton-air's
//! `ChallengeId` order (include/nhip_challenge_id.h), 59 sampled then the 4 that `Challenges::new`
//! derives.  Shared sub-circuits (`Rc` nodes) become one descriptor node each.  Any expression kind
//! not in the table fails the export (`ExportError::UnknownNode`): the verifier must never run a
//! circuit it did not receive whole.  `tests/test_air_export.py` checks the same mapping, written
//! in Python (`neptune_hip.air_export`), on hand-built circuits against the oracle's evaluator.
//!
//! Size: about 600 constraints over the master tables' 379 main / 88 aux columns (after degree
//! lowering); the descriptor's node count is the number of distinct sub-circuits, which the
//! verifier's slot compiler handles at any size (the triton-air-sized tests use ~22k nodes).
//!
//! Not compiled in the build container (no Rust toolchain, crates not vendored): the paths below
//! are triton-vm 1.0's public API; a mismatch there is a name to fix, not a change of design.
use std::cell::RefCell;
use std::collections::HashMap;
use std::rc::Rc;

use triton_constraint_builder::Constraints;
use triton_constraint_circuit::{
    BinOp, CircuitExpression, ConstraintCircuit, DualRowIndicator, InputIndicator, SingleRowIndicator,
};
use triton_vm::challenges::Challenges;
use triton_vm::table::master_table::{MasterAuxTable, MasterMainTable, MasterTable};

/// `0x41495231` ("AIR1"), the descriptor's magic word.
pub const AIR_MAGIC: u64 = 0x4149_5231;
pub const OP_INPUT: u64 = 0;
pub const OP_CONST: u64 = 1;
pub const OP_ADD: u64 = 2;
pub const OP_MUL: u64 = 4;
pub const IN_MAIN_CURR: u64 = 0;
pub const IN_AUX_CURR: u64 = 1;
pub const IN_MAIN_NEXT: u64 = 2;
pub const IN_AUX_NEXT: u64 = 3;
pub const IN_CHALLENGE: u64 = 4;

#[derive(Debug, Clone, PartialEq, Eq)]
pub enum ExportError {
    /// an expression kind the descriptor has no node for
    UnknownNode(String),
    /// a challenge index outside `ChallengeId`
    ChallengeIndex(usize),
    /// a column index outside the master table
    ColumnIndex { aux: bool, index: usize },
}

impl std::fmt::Display for ExportError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "AIR export: {self:?}")
    }
}
impl std::error::Error for ExportError {}

/// Maps an input indicator to (kind, column).
pub trait DescriptorInput: InputIndicator {
    fn kind_and_index(&self) -> (u64, usize);
}

impl DescriptorInput for SingleRowIndicator {
    fn kind_and_index(&self) -> (u64, usize) {
        match *self {
            SingleRowIndicator::Main(i) => (IN_MAIN_CURR, i),
            SingleRowIndicator::Aux(i) => (IN_AUX_CURR, i),
        }
    }
}

impl DescriptorInput for DualRowIndicator {
    fn kind_and_index(&self) -> (u64, usize) {
        match *self {
            DualRowIndicator::CurrentMain(i) => (IN_MAIN_CURR, i),
            DualRowIndicator::CurrentAux(i) => (IN_AUX_CURR, i),
            DualRowIndicator::NextMain(i) => (IN_MAIN_NEXT, i),
            DualRowIndicator::NextAux(i) => (IN_AUX_NEXT, i),
        }
    }
}

/// Accumulates descriptor nodes; one node per distinct `Rc` sub-circuit, keyed by address.  The
/// builder keeps a reference to every node it has keyed, so no address is freed and reused by
/// another circuit while it lives (the constraint groups' circuits are dropped between groups).
pub struct DescriptorBuilder {
    pub num_main: usize,
    pub num_aux: usize,
    pub num_challenges: usize,
    nodes: Vec<[u64; 4]>,
    memo: HashMap<usize, u64>,
    keep: Vec<Box<dyn std::any::Any>>,
}

impl DescriptorBuilder {
    pub fn new(num_main: usize, num_aux: usize, num_challenges: usize) -> Self {
        DescriptorBuilder { num_main, num_aux, num_challenges, nodes: Vec::new(), memo: HashMap::new(),
                            keep: Vec::new() }
    }

    fn push(&mut self, n: [u64; 4]) -> u64 {
        self.nodes.push(n);
        (self.nodes.len() - 1) as u64
    }

    fn leaf<II: DescriptorInput>(&mut self, e: &CircuitExpression<II>) -> Result<Option<[u64; 4]>, ExportError> {
        Ok(Some(match e {
            CircuitExpression::BConst(b) => [OP_CONST, b.value(), 0, 0],
            CircuitExpression::XConst(x) => {
                let c = x.coefficients;
                [OP_CONST, c[0].value(), c[1].value(), c[2].value()]
            }
            CircuitExpression::Input(ii) => {
                let (kind, idx) = ii.kind_and_index();
                let lim = if kind == IN_MAIN_CURR || kind == IN_MAIN_NEXT { self.num_main } else { self.num_aux };
                if idx >= lim {
                    return Err(ExportError::ColumnIndex { aux: kind == IN_AUX_CURR || kind == IN_AUX_NEXT, index: idx });
                }
                [OP_INPUT, kind, idx as u64, 0]
            }
            CircuitExpression::Challenge(i) => {
                if *i >= self.num_challenges {
                    return Err(ExportError::ChallengeIndex(*i));
                }
                [OP_INPUT, IN_CHALLENGE, *i as u64, 0]
            }
            CircuitExpression::BinOp(..) => return Ok(None),
            #[allow(unreachable_patterns)]
            other => return Err(ExportError::UnknownNode(format!("{other:?}"))),
        }))
    }

    /// The descriptor node id of `root`, adding its sub-circuits post-order (operands first) with
    /// an explicit stack (circuits are thousands of nodes deep after degree lowering).
    pub fn add<II: DescriptorInput + 'static>(&mut self, root: &Rc<RefCell<ConstraintCircuit<II>>>)
                                             -> Result<u64, ExportError> {
        let key = |r: &Rc<RefCell<ConstraintCircuit<II>>>| Rc::as_ptr(r) as usize;
        let mut stack: Vec<(Rc<RefCell<ConstraintCircuit<II>>>, bool)> = vec![(root.clone(), false)];
        while let Some((node, expanded)) = stack.pop() {
            if self.memo.contains_key(&key(&node)) {
                continue;
            }
            let circuit = node.borrow();
            match &circuit.expression {
                CircuitExpression::BinOp(op, a, b) => {
                    if !expanded {
                        stack.push((node.clone(), true));
                        stack.push((b.clone(), false));
                        stack.push((a.clone(), false));
                        continue;
                    }
                    let (ia, ib) = (self.memo[&key(a)], self.memo[&key(b)]);
                    let opc = match op {
                        BinOp::Add => OP_ADD,
                        BinOp::Mul => OP_MUL,
                        #[allow(unreachable_patterns)]
                        other => return Err(ExportError::UnknownNode(format!("{other:?}"))),
                    };
                    let id = self.push([opc, ia, ib, 0]);
                    self.memo.insert(key(&node), id);
                    self.keep.push(Box::new(node.clone()));
                }
                e => {
                    let n = self.leaf(e)?.expect("leaf");
                    let id = self.push(n);
                    self.memo.insert(key(&node), id);
                    self.keep.push(Box::new(node.clone()));
                }
            }
        }
        Ok(self.memo[&key(root)])
    }

    /// The descriptor: header, nodes, then the constraint node ids by type.
    pub fn finish(self, num_sampled: usize, groups: [Vec<u64>; 4]) -> Vec<u64> {
        let mut w = vec![AIR_MAGIC, self.num_main as u64, self.num_aux as u64, num_sampled as u64,
                         self.nodes.len() as u64];
        w.extend(groups.iter().map(|g| g.len() as u64));
        for n in &self.nodes {
            w.extend_from_slice(n);
        }
        for g in &groups {
            w.extend_from_slice(g);
        }
        w
    }
}

/// The constraints `triton_vm::verify` evaluates, as triton-vm's build script builds them.
pub fn triton_constraints() -> Constraints {
    let mut constraints = Constraints::all();
    let lowering = Constraints::default_degree_lowering_info();
    let substitutions = constraints.lower_to_target_degree_through_substitutions(lowering);
    constraints.combine_with_substitution_induced_constraints(substitutions)
}

fn group<II: DescriptorInput + 'static>(b: &mut DescriptorBuilder, cs: &[ConstraintCircuit<II>])
                              -> Result<Vec<u64>, ExportError> {
    // `Constraints::{init, cons, tran, term}()` hand out the consumed circuits; each constraint
    // is wrapped so the builder can key it like its shared operands
    cs.iter().map(|c| b.add(&Rc::new(RefCell::new(c.clone())))).collect()
}

/// The descriptor words of triton-air 1.0.0's constraints, for `nhip_air_create`
/// (`crate::Air::triton`).  Deterministic: the same words on every call.
pub fn triton_air_descriptor() -> Result<Vec<u64>, ExportError> {
    let c = triton_constraints();
    let mut b = DescriptorBuilder::new(MasterMainTable::NUM_COLUMNS, MasterAuxTable::NUM_COLUMNS,
                                       Challenges::COUNT);
    let init = group(&mut b, &c.init())?;
    let cons = group(&mut b, &c.cons())?;
    let tran = group(&mut b, &c.tran())?;
    let term = group(&mut b, &c.term())?;
    Ok(b.finish(Challenges::SAMPLE_COUNT, [init, cons, tran, term]))
}

#[cfg(test)]
mod tests {
    use super::*;

    #[test]
    fn challenge_layout_matches_the_descriptor_contract() {
        // include/nhip_challenge_id.h: 59 sampled + 4 derived, derived ones last
        assert_eq!(Challenges::SAMPLE_COUNT, 59);
        assert_eq!(Challenges::COUNT, 63);
        use triton_vm::air::challenge_id::ChallengeId;
        assert_eq!(ChallengeId::LookupTablePublicIndeterminate.index(), 54);
        assert_eq!(ChallengeId::StandardInputTerminal.index(), 59);
        assert_eq!(ChallengeId::CompressedProgramDigest.index(), 62);
    }

    #[test]
    fn descriptor_has_the_generated_evaluators_constraint_counts() {
        let w = triton_air_descriptor().unwrap();
        assert_eq!(w[0], AIR_MAGIC);
        assert_eq!((w[1] as usize, w[2] as usize, w[3]), (MasterMainTable::NUM_COLUMNS, MasterAuxTable::NUM_COLUMNS, 59));
        assert_eq!(w[5] as usize, MasterAuxTable::NUM_INITIAL_CONSTRAINTS);
        assert_eq!(w[6] as usize, MasterAuxTable::NUM_CONSISTENCY_CONSTRAINTS);
        assert_eq!(w[7] as usize, MasterAuxTable::NUM_TRANSITION_CONSTRAINTS);
        assert_eq!(w[8] as usize, MasterAuxTable::NUM_TERMINAL_CONSTRAINTS);
        assert_eq!(w.len(), 9 + 4 * w[4] as usize + (w[5] + w[6] + w[7] + w[8]) as usize);
        assert_eq!(triton_air_descriptor().unwrap(), w); // deterministic
    }
}
