/* sync_converge.c -- how far a speculative Huffman decode started at a random bit (assuming MCU block 0)
 * runs before it merges with the true decode: bit-position sync vs full (position + MCU phase) sync.
 * build: gcc -O2 -w -o /tmp/sync_converge tools/sync_converge.c -lm ; run: /tmp/sync_converge img.jpg */
#include "../oracle/sdsj_oracle.c"  /* test infrastructure: the oracle's parser and tables */
#include <stdio.h>
// unstuffed stream bit reader (no restarts)
static uint8_t *U; static size_t UN;
static int getb(uint64_t p, int n){ uint32_t v=0; for(int i=0;i<n;i++){uint64_t q=p+i; int bit = q/8<UN ? (U[q/8]>>(7-q%8))&1 : 0; v=(v<<1)|bit;} return v; }
static int hdec(uint64_t *p, const htable_t *t){ int l=1; int code=getb(*p,1); (*p)++; while(code>t->maxcode[l]){ code=(code<<1)|getb(*p,1); (*p)++; l++; if(l>16) return 0;} return t->vals[(code+t->valoffset[l])&0xFF]; }
int blkcomp[10], bpm;
// decode one block starting at p with component c; returns new p
static uint64_t dblock(uint64_t p, jpeg_t *j, int c){ comp_t *cp=&j->comp[c]; int s=hdec(&p,&j->dc[cp->td]); if(s>16) s=16; p+=s; for(int k=1;k<64;k++){int sym=hdec(&p,&j->ac[cp->ta]); int r=sym>>4; s=sym&15; if(s){k+=r; p+=s;} else { if(r!=15) break; k+=15;}} return p; }
int main(int argc,char**argv){
  FILE*f=fopen(argv[1],"rb"); static uint8_t d[1<<24]; size_t n=fread(d,1,sizeof d,f); fclose(f);
  jpeg_t j; memset(&j,0,sizeof j); if(parse_headers(d,n,&j)||setup_geometry(&j)){printf("parse fail\n");return 1;}
  U=malloc(n); UN=0; for(size_t i=j.entropy_off;i<n;i++){ if(d[i]==0xFF){ if(d[i+1]==0){U[UN++]=0xFF;i++;continue;} else break;} U[UN++]=d[i]; }
  bpm=0; for(int c=0;c<j.ncomp;c++) for(int k=0;k<j.comp[c].h*j.comp[c].v;k++) blkcomp[bpm++]=c;
  int total=j.mcux*j.mcuy*bpm; uint64_t *bs=malloc(sizeof(uint64_t)*(total+1)); uint64_t p=0;
  // map bitpos -> block index+1 via hash array
  int *at = calloc(UN*8+64, sizeof(int));
  for(int b=0;b<total;b++){ bs[b]=p; at[p]=b+1; p=dblock(p,&j,blkcomp[b%bpm]); }
  printf("bits=%llu blocks=%d bits/block=%.1f\n",(unsigned long long)p,total,(double)p/total);
  int W = argc>2?atoi(argv[2]):0;
  srand(7); int N=2000; long long sumb=0, sumblk=0; int hist[12]={0}; int maxb=0; long long possync=0;
  for(int t=0;t<N;t++){ uint64_t s=(uint64_t)((double)rand()/RAND_MAX*(p-20000)); uint64_t q=s; int ph=0; int nb=0; int firstpos=-1;
    for(;;){ if(at[q]){ int b=at[q]-1; if(firstpos<0) firstpos=q-s; if(b%bpm==ph) break;} q=dblock(q,&j,blkcomp[ph]); ph=(ph+1)%bpm; nb++; if(q>=p) break; }
    int dist=(int)(q-s); sumb+=dist; sumblk+=nb; if(dist>maxb)maxb=dist; possync+=firstpos; int h=0; while((512<<h)<dist && h<11) h++; hist[h]++; }
  printf("mean bits to full sync=%.0f blocks=%.1f max=%d ; mean bits to first pos-sync=%.0f\n",(double)sumb/N,(double)sumblk/N,maxb,(double)possync/N);
  for(int h=0;h<12;h++) printf("<=%d: %d\n",512<<h,hist[h]);
}
