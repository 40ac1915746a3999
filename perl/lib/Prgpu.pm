package Prgpu;

# Perl side of the XS binding (perl/Prgpu.xs) of libprgpu: the consensus stage
# (run_chunk), the seed-extension stage (mem), one whole iteration (iteration) and the
# per-iteration masking (mask).
#
# Consensus: what a proovread maintainer calls instead of fanning bam2cns out over xargs
# (bin/proovread:1596-1619): one Prgpu::run_chunk per chunk of long reads, with the
# reads' SAM records in BAM order.  The record fields read here are the ones the
# Sam::Seq engine reads (Sam/Alignment.pm:87-110: POS, CIGAR, SEQ, QUAL, AS:i); the
# chunk is flattened into the SoA buffers of pr_cns_batch (include/prgpu.h) with pack,
# the same layout proovread_amd/cns.py:pack_chunk builds.
#
#   my $ctx = Prgpu::Context->new(0);
#   my @res = Prgpu::run_chunk($ctx, {coverage => 11.25, use_ref_qual => 1},
#                              [{id => 'r1', seq => $seq, qual => $qual, desc => $desc}],
#                              [[@sam_lines_of_r1]]);
#   print Prgpu::fastq($_) for @res;            # bam2cns:453
#   print Prgpu::chim_lines($_) for @res;       # bam2cns:488
#
# There is no CPU fallback: without a gfx950 device Context->new dies.

use strict;
use warnings;

our $VERSION = '0.1';

require XSLoader;
XSLoader::load('Prgpu', $VERSION);

# status codes of include/prgpu.h
our %ERRORS = (0 => 'PR_OK', -1 => 'PR_ERR_ARG', -2 => 'PR_ERR_HIP', -3 => 'PR_ERR_SAM',
               -4 => 'PR_ERR_NOSEQ', -5 => 'PR_ERR_BIN_RANGE', -6 => 'PR_ERR_DIV0',
               -7 => 'PR_ERR_CIGAR', -8 => 'PR_ERR_BEYOND_REF', -9 => 'PR_ERR_CAPACITY',
               -10 => 'PR_ERR_UNSUPPORTED');

my %CIGAR_OP = (M => 0, I => 1, D => 2, N => 3, S => 4, H => 5, P => 6, '=' => 7, X => 8);
use constant { ALN_HAS_SCORE => 1, ALN_NO_QUAL => 2, ALN_NO_SEQ => 4 };

package Prgpu::Context;

sub new {
    my ($class, $device) = @_;
    my $h = Prgpu::ctx_create(defined $device ? $device : 0);
    return bless {h => $h}, $class;
}

sub handle { $_[0]{h} }

sub DESTROY {
    my $self = shift;
    Prgpu::ctx_destroy($self->{h}) if $self->{h};
    $self->{h} = 0;
}

package Prgpu;

# CIGAR string -> BAM-coded ops (len<<4 | op); dies on a malformed string like
# Sam::Alignment's cigar parsing would produce garbage for
sub cigar_ops {
    my ($cig) = @_;
    return () if $cig eq '*';
    my @ops;
    my $rest = $cig;
    while ($rest =~ s/^(\d+)([MIDNSHP=X])//) {
        push @ops, ($1 << 4) | $CIGAR_OP{$2};
    }
    die "Prgpu: bad CIGAR '$cig'\n" if length $rest;
    return @ops;
}

# Flatten reads + SAM records into the packed fields of pr_cns_batch.
sub pack_chunk {
    my ($reads, $alns) = @_;
    my $n = @$reads;
    my %b = (n_lr => $n);
    my $has_ref = $n > 0;
    for my $r (@$reads) { $has_ref = 0 unless defined $r->{seq} }
    my (@lr_off, @ign_off, @ign) = (0);
    my ($ref_seq, $ref_qual) = ('', '');
    my $any_ign = 0;
    @ign_off = (0);
    for my $r (@$reads) {
        my $len = defined $r->{seq} ? length($r->{seq}) : $r->{length};
        push @lr_off, $lr_off[-1] + $len;
        if ($has_ref) {
            $ref_seq .= $r->{seq};
            # a quality string shorter than the sequence contributes nothing past its end
            # (Seq.pm:262 `next unless $freqs[$i]`): pad with phred 0
            my $q = defined $r->{qual} ? substr($r->{qual}, 0, $len) : '';
            $ref_qual .= $q . ('!' x ($len - length $q));
            # bam2cns:382-391: MCRn:off,len tags of the reference description
            my @m = (($r->{desc} // '') =~ /MCR\d+:(\d+),(\d+)/g);
            $any_ign ||= @m;
            push @ign, @m;
        }
        push @ign_off, @ign / 2;
    }
    $b{lr_off} = pack('q<*', @lr_off);
    if ($has_ref) {
        $b{ref_seq} = $ref_seq;
        $b{ref_qual} = $ref_qual;
    }
    if ($any_ign) {
        $b{ign_off} = pack('q<*', @ign_off);
        $b{ign} = pack('l<*', @ign);
    }
    my (@aln_off, @pos, @score, @flags, @seq_off, @lseq, @cig_off, @ncig, @cig) = (0);
    my ($seq_pool, $qual_pool) = ('', '');
    for my $list (@$alns) {
        for my $line (@$list) {
            chomp(my $l = $line);
            my @f = split /\t/, $l, 12;
            die "Prgpu: SAM line with < 11 fields\n" if @f < 11;
            my $fl = 0;
            my $sc = 0;
            if (@f == 12) {
                for my $t (split /\t/, $f[11]) {
                    if (substr($t, 0, 2) eq 'AS') {
                        no warnings 'numeric';
                        $sc = 0 + substr($t, 5);   # Perl's own numification, as Sam::Alignment
                        $fl |= ALN_HAS_SCORE;
                    }
                }
            }
            my $s = $f[9] eq '*' ? '' : $f[9];
            $fl |= ALN_NO_SEQ if $f[9] eq '*';
            my $q;
            if ($f[10] eq '*') {
                $fl |= ALN_NO_QUAL;
                $q = '!' x length $s;
            } else {
                $q = substr($f[10], 0, length $s);
                $q .= '!' x (length($s) - length $q);
            }
            my @ops = cigar_ops($f[5]);
            push @pos, $f[3];
            push @score, $sc;
            push @flags, $fl;
            push @seq_off, length $seq_pool;
            push @lseq, length $s;
            push @cig_off, scalar @cig;
            push @ncig, scalar @ops;
            push @cig, @ops;
            $seq_pool .= $s;
            $qual_pool .= $q;
        }
        push @aln_off, scalar @pos;
    }
    $b{aln_off} = pack('q<*', @aln_off);
    $b{aln_pos} = pack('l<*', @pos);
    $b{aln_score} = pack('d<*', @score);
    $b{aln_flags} = pack('C*', @flags);
    $b{aln_seq_off} = pack('q<*', @seq_off);
    $b{aln_lseq} = pack('l<*', @lseq);
    $b{aln_cig_off} = pack('q<*', @cig_off);
    $b{aln_ncig} = pack('l<*', @ncig);
    $b{seq_pool} = $seq_pool;
    $b{qual_pool} = $qual_pool;
    $b{cig_pool} = pack('L<*', @cig);
    return \%b;
}

# One bam2cns chunk on the GPU (bam2cns:332-365 for every read).  Returns one hash per
# read: id, status (0 or a PR_ERR_* code), seq, qual, trace, cigar (string), chim
# ([from, to, n_pos, n_cols] records).
sub run_chunk {
    my ($ctx, $params, $reads, $alns) = @_;
    die "Prgpu::run_chunk: reads and alignment lists differ in length\n" unless @$reads == @$alns;
    my $b = pack_chunk($reads, $alns);
    my $o = cns_run(ref $ctx ? $ctx->handle : $ctx, $params, $b);
    return cns_results($o, [map { $_->{id} } @$reads]);
}

# per-read results of a packed consensus output (cns_run / iter_run)
sub cns_results {
    my ($o, $ids) = @_;
    my $n = @$ids;
    my @off = unpack('q<*', $o->{out_off});
    my @st = unpack('l<*', $o->{status});
    my @sl = unpack('l<*', $o->{seq_len});
    my @tl = unpack('l<*', $o->{trace_len});
    my @nc = unpack('l<*', $o->{ncigar});
    my @nch = unpack('l<*', $o->{nchim});
    my @choff = unpack('q<*', $o->{chim_off});
    my @res;
    for my $i (0 .. $n - 1) {
        my %r = (id => $ids->[$i], status => $st[$i]);
        if ($st[$i] == 0) {
            my $p = $off[$i];
            $r{seq} = substr($o->{seq}, $p, $sl[$i]);
            $r{qual} = substr($o->{qual}, $p, $sl[$i]);
            $r{trace} = substr($o->{trace}, $p, $tl[$i]);
            $r{cigar} = join '', map { ($_ >> 4) . substr('MID', $_ & 15, 1) }
                unpack('L<*', substr($o->{cigar}, 4 * $p, 4 * $nc[$i]));
            my @c = unpack('l<*', substr($o->{chim}, 16 * $choff[$i], 16 * $nch[$i]));
            $r{chim} = [map { [@c[4 * $_ .. 4 * $_ + 3]] } 0 .. $nch[$i] - 1];
        }
        push @res, \%r;
    }
    return @res;
}

# ------------------------------------------------------------------ seed-extension stage
#
# What bin/proovread's run_bwa (bin/proovread:1254-1322) gets from a `bwa-proovread mem -a -Y`
# process: SAM records of every short read against the long reads, here from the library's
# seeding front end (seed_index_build / seed_map, host) and the GPU seed extension (sw_run),
# with the records written the way proovread_amd/bwa_proovread.py:mem writes them.

my @NT = ('A', 'C', 'G', 'T', 'N');
my $CIGAR_CHARS = 'MIDNSHP=X';

# bwa's nst_nt4_table: A C G T (either case) -> 0..3, everything else -> 4
sub nt4 {
    my ($s) = @_;
    $s =~ tr/ACGTacgt/\x04/c;
    $s =~ tr/ACGTacgt/\x00\x01\x02\x03\x00\x01\x02\x03/;
    return $s;
}

# sequences -> (nt4 pool, packed int64 offsets)
sub pool {
    my ($seqs) = @_;
    my @off = (0);
    push @off, $off[-1] + length $_ for @$seqs;
    return (nt4(join '', @$seqs), pack('q<*', @off));
}

use constant TASK_BYTES => 40;   # pr_seed_task: 10 x int32

# SW results of a packed sw_run output for tasks 0..n-1
sub sw_unpack {
    my ($o, $n) = @_;
    my @co = unpack('q<*', $o->{cigar_off});   # variable-length CIGARs, compacted in task order
    my @cig;
    for my $t (0 .. $n - 1) {
        my @ops = unpack('L<*', substr($o->{cigar}, 4 * $co[$t], 4 * ($co[$t + 1] - $co[$t])));
        push @cig, join '', map { ($_ >> 4) . substr($CIGAR_CHARS, $_ & 15, 1) } @ops;
    }
    return {pos => [unpack('l<*', $o->{pos})], score => [unpack('l<*', $o->{score})],
            pass => [unpack('C*', $o->{pass})], status => [unpack('l<*', $o->{status})], cigar => \@cig,
            task => [unpack('l<*', $o->{task})], flag => [unpack('l<*', $o->{flag})]};
}

# Sam::Alignment::length (Alignment.pm:417-431): M+D if SEQ is empty or the CIGAR starts or
# ends with S, else the SEQ length
sub aln_length {
    my ($cig, $seq_len) = @_;
    my @ops = $cig =~ /(\d+)([MIDNSHP=X])/g;
    if ($seq_len == 0 || (@ops && ($ops[1] eq 'S' || $ops[-1] eq 'S'))) {
        my $l = 0;
        for (my $i = 0; $i < @ops; $i += 2) { $l += $ops[$i] if $ops[$i + 1] eq 'M' || $ops[$i + 1] eq 'D' }
        return $l;
    }
    return $seq_len;
}

# Host seeding of sr_seqs against lr_seqs (seed_index_build / seed_map) -> the pr_sw_batch
# fields (nt4 pools, offsets, task columns in read order, chain order) and the task columns.
sub seed_batch {
    my (%a) = @_;
    my ($lr_pool, $lr_off) = pool($a{lr_seqs});
    my ($sr_pool, $sr_off) = pool($a{sr_seqs});
    my $ix = seed_index_build($lr_pool, $lr_off);
    my $packed = eval { seed_map($ix, $a{seed_opts} || {}, $sr_pool, $sr_off, $a{threads} || 0) };
    my $err = $@;
    seed_index_free($ix);
    die $err if $err;
    my $nt = length($packed) / TASK_BYTES;
    my (@t_sr, @t_lr, @t_strand, @t_qbeg, @t_rbeg, @t_slen, @t_chain);
    for my $t (0 .. $nt - 1) {
        my @f = unpack('l<10', substr($packed, TASK_BYTES * $t, TASK_BYTES));
        push @t_sr, $f[0];
        push @t_lr, $f[1];
        push @t_strand, $f[2];
        push @t_qbeg, $f[3];
        push @t_rbeg, $f[4];
        push @t_slen, $f[5];
        push @t_chain, $f[8];
    }
    # bwa mode: every seed of the kept chains, grouped by short read, then chain (t_chain)
    my %batch = (sr_seq => $sr_pool, sr_off => $sr_off, lr_seq => $lr_pool, lr_off => $lr_off, n_task => $nt,
                 t_sr => pack('l<*', @t_sr), t_lr => pack('l<*', @t_lr), t_strand => pack('C*', @t_strand),
                 t_qbeg => pack('l<*', @t_qbeg), t_rbeg => pack('l<*', @t_rbeg), t_slen => pack('l<*', @t_slen),
                 t_chain => pack('l<*', @t_chain));
    return (\%batch, {sr => \@t_sr, lr => \@t_lr, strand => \@t_strand, qbeg => \@t_qbeg, rbeg => \@t_rbeg,
                      slen => \@t_slen, chain => \@t_chain});
}

# names -> (concatenated names, packed int64 offsets)
sub names_pool {
    my ($names) = @_;
    my @off = (0);
    push @off, $off[-1] + length $_ for @$names;
    return (join('', @$names), pack('q<*', @off));
}

# mem(%a) -> (header lines, record lines): the output of `bwa-proovread mem`.
#   ctx        Prgpu::Context: the whole of mem on the device (mem_gpu: the index and the seeds in
#              HBM, bwa mode, the -b/-l filter on the device, the records formatted in the
#              library); or a sw_runner coderef taking the host seeding's batch hash and returning
#              {pos, score, pass, status, cigar, task, flag} arrays per reported alignment in SAM
#              order — the tests inject the oracle; the records are then formatted here)
#   seed_opts, sw_opts  option hashes for seed_map / sw_run ({finish => 0|1, ...})
#   b, l       the -b/-l bin filter (0: off)
#   threads    host seeding threads
#   lr_names, lr_seqs, sr_names, sr_seqs, sr_quals (undef entries for FASTA reads)
#   cl         the command line for @PG
sub mem {
    my (%a) = @_;
    if (ref $a{ctx} ne 'CODE') {
        my @head = ("\@HD\tVN:1.5\tSO:unsorted\n");
        push @head, "\@SQ\tSN:$a{lr_names}[$_]\tLN:" . length($a{lr_seqs}[$_]) . "\n" for 0 .. $#{$a{lr_names}};
        push @head, "\@PG\tID:bwa-proovread\tPN:bwa-proovread\tVN:prgpu\tCL:bwa-proovread mem " . ($a{cl} // '') . "\n";
        my ($lr_pool, $lr_off) = pool($a{lr_seqs});
        my ($sr_pool, $sr_off) = pool($a{sr_seqs});
        my ($srn, $srn_off) = names_pool($a{sr_names});
        my ($lrn, $lrn_off) = names_pool($a{lr_names});
        my %in = (sr_seq => $sr_pool, sr_off => $sr_off, lr_seq => $lr_pool, lr_off => $lr_off,
                  sr_text => join('', @{$a{sr_seqs}}), sr_names => $srn, sr_name_off => $srn_off, lr_names => $lrn,
                  lr_name_off => $lrn_off, b => $a{b} || 0, l => $a{l} || 0, threads => $a{threads} || 0);
        my $quals = $a{sr_quals} || [];
        $in{sr_qual} = join('', @$quals) if @$quals == @{$a{sr_seqs}} && !grep { !defined } @$quals;
        my $text = mem_gpu(ref $a{ctx} ? $a{ctx}->handle : $a{ctx}, $a{seed_opts} || {}, $a{sw_opts} || {}, \%in);
        my @rec = split /(?<=\n)/, $text;
        return (\@head, \@rec);
    }
    my ($bt, $tc) = seed_batch(%a);
    my %batch = %$bt;
    my $nt = $batch{n_task};
    my ($t_sr, $t_lr, $t_strand) = @$tc{qw(sr lr strand)};
    my @t_sr = @$t_sr;
    my @t_lr = @$t_lr;
    my @t_strand = @$t_strand;
    my $res;
    if (ref $a{ctx} eq 'CODE') {
        $res = $a{ctx}->(\%batch);
    } else {
        my $o = sw_run(ref $a{ctx} ? $a{ctx}->handle : $a{ctx}, $a{sw_opts} || {}, \%batch);
        $res = sw_unpack($o, $o->{n});
    }


    my @head = ("\@HD\tVN:1.5\tSO:unsorted\n");
    push @head, "\@SQ\tSN:$a{lr_names}[$_]\tLN:" . length($a{lr_seqs}[$_]) . "\n" for 0 .. $#{$a{lr_names}};
    push @head, "\@PG\tID:bwa-proovread\tPN:bwa-proovread\tVN:prgpu\tCL:bwa-proovread mem " . ($a{cl} // '') . "\n";

    # -b/-l binning: Sam::Seq add_aln_by_score over the run's records (bwa_proovread.py BinFilter)
    my (%bins, @alive);
    my $filter = ($a{b} || 0) > 0 && ($a{l} || 0) > 0;
    my $bin_add = sub {
        my ($lr, $pos1, $len, $score) = @_;
        my $rid = @alive;
        push @alive, 0;
        return if $len <= 0;
        my $nc = ($score / $len) * ($len / (40 + $len));
        my $ent = $bins{$lr, int(($pos1 + $len / 2.0) / $a{b})} ||= [0, []];
        my $lst = $ent->[1];
        if ($ent->[0] > $a{l}) {
            return if $nc <= $lst->[-1][0];
            my $old = pop @$lst;
            $alive[$old->[1]] = 0;
            $ent->[0] -= $old->[2];
        }
        $ent->[0] += $len;
        my $i = $#$lst;
        --$i while $i >= 0 && $nc > $lst->[$i][0];
        splice @$lst, $i + 1, 0, [$nc, $rid, $len];
        $alive[$rid] = 1;
    };

    # the reported alignments in SAM order, read by read (bwa mode: the device ran mem_chain2aln,
    # mem_sort_dedup_patch, mem_mark_primary_se and mem_reg2sam's filters)
    my @rec;
    my ($pos, $sc, $ps, $st, $cg, $tk, $fl) = @$res{qw(pos score pass status cigar task flag)};
    for my $i (0 .. $#$pos) {
        next unless $st->[$i] == 0 && $ps->[$i];
        my $x = $tk->[$i];
        my $r = $t_sr[$x];
        my $strand = $t_strand[$x];
        my $q = $a{sr_seqs}[$r];
        my $qual = $a{sr_quals}[$r];
        my ($s, $qq);
        if ($strand) {
            ($s = $q) =~ tr/ACGTacgt/N/c;
            $s =~ tr/ACGTacgt/TGCATGCA/;
            $s = reverse $s;
            $qq = defined $qual ? scalar reverse($qual) : '*';
        } else {
            $s = uc $q;
            $qq = defined $qual ? $qual : '*';
        }
        my $flag = $fl->[$i];
        my $mapq = $flag & 0x100 ? 0 : 60;   # mem_approx_mapq_se is not restated
        push @rec, join("\t", $a{sr_names}[$r], $flag, $a{lr_names}[$t_lr[$x]], $pos->[$i] + 1, $mapq,
                        $cg->[$i], '*', 0, 0, $s, $qq, "AS:i:$sc->[$i]") . "\n";
        $bin_add->($t_lr[$x], $pos->[$i] + 1, aln_length($cg->[$i], length $q), $sc->[$i]) if $filter;
    }
    @rec = @rec[grep { $alive[$_] } 0 .. $#rec] if $filter;
    return (\@head, \@rec);
}

# ------------------------------------------------------------------ one iteration in one call
#
# iteration(%a): one proovread correction task (bin/proovread:835-869: bwa-proovread mem,
# samtools sort, the bam2cns fan-out) on the device without SAM/BAM files: host seeding of
# sr_seqs against lr_seqs, then iter_run (seed extension + CIGAR, hand-off in samtools
# coordinate order, consensus of every long read).  Returns run_chunk-style per-read results.
#   ctx, seed_opts, sw_opts, threads   as for mem
#   params     consensus options as for run_chunk
#   lr_ids, lr_seqs (the mapping reference: the previous task's .masked.fa from the second
#   iteration on), lr_quals (default phred 3 '$', raw CLR reads), ref_seqs (the consensus
#   reference, the previous task's unmasked .fq; default lr_seqs), sr_seqs
sub iteration {
    my (%a) = @_;
    if (ref $a{ctx} ne 'CODE') {   # the seeding on the device too (iter_run_gpu)
        my ($lr_pool, $lr_off) = pool($a{lr_seqs});
        my ($sr_pool, $sr_off) = pool($a{sr_seqs});
        my %batch = (sr_seq => $sr_pool, sr_off => $sr_off, lr_seq => $lr_pool, lr_off => $lr_off);
        $batch{lr_qual} = join '', map {
            my $q = $a{lr_quals} ? $a{lr_quals}[$_] : undef;
            defined $q ? $q : '$' x length $a{lr_seqs}[$_]
        } 0 .. $#{$a{lr_seqs}};
        $batch{ref_seq} = join '', @{$a{ref_seqs}} if $a{ref_seqs};
        my $o = iter_run_gpu(ref $a{ctx} ? $a{ctx}->handle : $a{ctx}, $a{seed_opts} || {}, $a{sw_opts} || {},
                             $a{params} || {}, \%batch);
        return cns_results($o, $a{lr_ids});
    }
    my ($bt, $tc) = seed_batch(%a);
    my %batch = %$bt;   # bwa mode: the seeds as pr_seed_map returns them, grouped on the device
    $batch{lr_qual} = join '', map {
        my $q = $a{lr_quals} ? $a{lr_quals}[$_] : undef;
        defined $q ? $q : '$' x length $a{lr_seqs}[$_]
    } 0 .. $#{$a{lr_seqs}};
    $batch{ref_seq} = join '', @{$a{ref_seqs}} if $a{ref_seqs};
    my $o = ref $a{ctx} eq 'CODE' ? $a{ctx}->(\%batch)
          : iter_run(ref $a{ctx} ? $a{ctx}->handle : $a{ctx}, $a{sw_opts} || {}, $a{params} || {}, \%batch);
    return cns_results($o, $a{lr_ids});
}

# ------------------------------------------------------------------ masking
#
# `SeqFilter --phred-mask <hcr-mask> --base-content N` after every iteration (bin/proovread:1701-1716)
# on the GPU: mask($ctx, hcr_mask => '20,41,80,130,60,0.7', min_sr_length => 150,
# seqs => [...], quals => [...]) -> (\@masked, \@mcrs ([[off, len], ...] per read), [bpt, bpN]);
# bpN / bpt is the input of mask_shortcut_frac (bin/proovread:2026-2047).
sub mask {
    my ($ctx, %a) = @_;
    my $p = mask_params($a{hcr_mask} // '20,41,80,130,60,0.7', $a{min_sr_length} // 100);
    $p->{phred_offset} = $a{phred_offset} if defined $a{phred_offset};
    my ($seqs, $quals) = @a{qw(seqs quals)};
    die "Prgpu::mask: every read needs a quality string of its length\n"
        if @$seqs != @$quals || grep { length $seqs->[$_] != length $quals->[$_] } 0 .. $#$seqs;
    my @off = (0);
    push @off, $off[-1] + length $_ for @$seqs;
    my $o = mask_run(ref $ctx ? $ctx->handle : $ctx, $p, join('', @$seqs), join('', @$quals), pack('q<*', @off));
    my @moff = unpack('q<*', $o->{mcr_off});
    my @nm = unpack('l<*', $o->{n_mcr});
    my (@masked, @mcrs);
    for my $i (0 .. $#$seqs) {
        push @masked, substr($o->{seq}, $off[$i], $off[$i + 1] - $off[$i]);
        my @v = unpack('l<*', substr($o->{mcr}, 8 * $moff[$i], 8 * $nm[$i]));
        push @mcrs, [map { [@v[2 * $_, 2 * $_ + 1]] } 0 .. $nm[$i] - 1];
    }
    return (\@masked, \@mcrs, [unpack('q<2', $o->{stats})]);
}

# the FASTQ record bam2cns prints (bam2cns:453, Fastq::Seq string)
sub fastq {
    my ($r) = @_;
    return "\@$r->{id}\n$r->{seq}\n+\n$r->{qual}\n";
}

# the .chim.tsv lines (bam2cns:488: printf "%s\t%d\t%d\t%s\n", score in Perl's own
# number stringification)
sub chim_lines {
    my ($r) = @_;
    return map { sprintf("%s\t%d\t%d\t%s\n", $r->{id}, $_->[0], $_->[1], $_->[2] / $_->[3]) } @{$r->{chim} || []};
}

1;
